set -o pipefail
o=gpurun_out/r2rot3; mkdir -p $o
for t in 15 16 17 99; do
for k in 0.7 1.0; do
LC_PLAN_K=$k LC_TEAM_ROT_LB=$t timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_t${t}_k$k.json 2> $o/c3_t${t}_k$k.err || exit 1
done
done
timeout -k 10 120 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > $o/c4.json 2> $o/c4.err || exit 1
timeout -k 10 120 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2.json 2> $o/c2.err || exit 1
echo done
