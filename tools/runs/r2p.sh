set -o pipefail
o=gpurun_out/r2p; mkdir -p $o
B="python -u bench.py --no-cpu --e2e-reps 0"
for k in 1 1.3 1.6 2.0 2.5; do
  LC_PLAN_K=$k timeout -k 10 120 $B --steps 10 --warmup 3 > $o/c3_k$k.json 2> /dev/null || exit 1
  LC_PLAN_K=$k timeout -k 10 120 $B --steps 10 --warmup 3 --emulate 2/8 > $o/e2_k$k.json 2> /dev/null || exit 1
done
LC_PLAN_K=1.6 LC_DEBUG=1 timeout -k 10 120 $B --steps 1 --warmup 1 > /dev/null 2> $o/c3_dbg_k1.6.err || exit 1
echo done
