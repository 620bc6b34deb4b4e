set -o pipefail
o=gpurun_out/r2x; mkdir -p $o
for k in 0.3 0.5 0.6 0.7 0.8; do
for w in 13 14; do
LC_MID_MAXW=$w LC_PLAN_K=$k LC_PIPE=207 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_w${w}_k$k.json 2> $o/c3_w${w}_k$k.err || exit 1
done
done
echo done
