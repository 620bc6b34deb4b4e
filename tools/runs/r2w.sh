set -o pipefail
o=gpurun_out/r2w; mkdir -p $o
for k in 0.7 1.0 1.3; do
for pp in 79 207; do
LC_MID_MAXW=14 LC_PLAN_K=$k LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_${pp}_k$k.json 2> $o/c3_${pp}_k$k.err || exit 1
done
done
echo done
