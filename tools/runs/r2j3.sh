set -o pipefail
o=gpurun_out/r2j3; mkdir -p $o
for k in 0.35 0.45 0.6; do
LC_PLAN_K=$k timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_k$k.json 2> /dev/null || exit 1
done
for m in 13 14; do
LC_MID_MAXW=$m timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_mid$m.json 2> /dev/null || exit 1
done
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c3_dbg.err || exit 1
echo done
