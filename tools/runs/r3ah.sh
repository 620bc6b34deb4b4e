set -o pipefail
# r3ah: the team model's cost per team bit (LC_PLAN_X, default 1.57) lowered so the planner may
# take tiles below 13 slots (LC_PLAN_LBMIN=11): C2, C4, C3 and the 8-way C3 shares
o=gpurun_out/r3ah; mkdir -p $o
export LC_PLAN_LBMIN=11
for x in 1.2 0.9; do
export LC_PLAN_X=$x
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c2 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c2_x${x}_dbg.log || exit 1
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c4_x${x}_dbg.log || exit 1
timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_x$x.json 2> $o/c2_x$x.log || exit 1
timeout -k 10 200 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4_x$x.json 2> $o/c4_x$x.log || exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_x$x.json 2> $o/c3_x$x.log || exit 1
for r in 0 1 2 3 4 5 6 7; do
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --emulate $r/8 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 >> $o/c3e_x$x.json 2>> $o/c3e_x$x.log || exit 1
done
echo "variant $x done"
done
echo done
