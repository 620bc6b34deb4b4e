set -o pipefail
o=gpurun_out/r2rf2; mkdir -p $o
for f in 0.6 0.8 1.0; do
for k in 0.4 0.45 0.5; do
LC_ROT_F=$f LC_PLAN_K=$k timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_f${f}_k$k.json 2> /dev/null || exit 1
done
done
echo done
