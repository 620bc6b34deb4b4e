set -o pipefail
o=gpurun_out/r2y2; mkdir -p $o
for rot in 0 2 5; do
LC_TEAM_ROT=$rot timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_rot$rot.json 2> /dev/null || exit 1
done
for lb in 13 14; do
LC_TEAM_ROT_LB=$lb timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_rlb$lb.json 2> /dev/null || exit 1
for r in 3 5; do
LC_TEAM_ROT_LB=$lb timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_rlb$lb.json 2> /dev/null || exit 1
done
done
echo done
