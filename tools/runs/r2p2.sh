set -o pipefail
o=gpurun_out/r2p2; mkdir -p $o
for k in 0.45 0.55 0.7 0.9; do
LC_PLAN_K=$k timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_k$k.json 2> /dev/null || exit 1
done
LC_PLAN_K=0.7 LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c3_k0.7_dbg.err || exit 1
echo done
