set -o pipefail
# r3ag: the team planner's smallest tile 13 (default) vs 12 / 11 slots (LC_PLAN_LBMIN): C2, C4, C3, 8-way C3 shares
o=gpurun_out/r3ag; mkdir -p $o
for v in 13 12 11; do
export LC_PLAN_LBMIN=$v
timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_m$v.json 2> $o/c2_m$v.log || exit 1
timeout -k 10 200 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4_m$v.json 2> $o/c4_m$v.log || exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_m$v.json 2> $o/c3_m$v.log || exit 1
for r in 0 1 2 3 4 5 6 7; do
timeout -k 10 200 python -u bench.py --emulate $r/8 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 >> $o/c3e_m$v.json 2>> $o/c3e_m$v.log || exit 1
done
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c4_m${v}_dbg.log || exit 1
echo "variant $v done"
done
echo done
