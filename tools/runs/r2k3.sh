set -o pipefail
o=gpurun_out/r2k3; mkdir -p $o
for rep in 1 2; do
for k in 0.45 0.6 0.75; do
for m in 13 14; do
LC_PLAN_K=$k LC_MID_MAXW=$m timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_k${k}_m${m}_$rep.json 2> /dev/null || exit 1
done
done
done
echo done
