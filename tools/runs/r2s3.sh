set -o pipefail
o=gpurun_out/r2s3; mkdir -p $o
for bh in 600 400; do
for s in 0/2 1/2; do
n=$(echo $s | tr / _)
LC_BATCH_HIST=$bh timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $s > $o/e${n}_bh$bh.json 2> /dev/null || exit 1
done
done
echo done
