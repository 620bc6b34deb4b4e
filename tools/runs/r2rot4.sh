set -o pipefail
o=gpurun_out/r2rot4; mkdir -p $o
for k in 0.4 0.5 0.6 0.7 0.8 0.9; do
LC_PLAN_K=$k timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_k$k.json 2> $o/c3_k$k.err || exit 1
done
for r in 0 1 2 3 4 5 6 7; do
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e$r.json 2> $o/e$r.err || exit 1
done
echo done
