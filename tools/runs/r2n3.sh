set -o pipefail
o=gpurun_out/r2n3; mkdir -p $o
for pb in 1 0; do
for s in 0/2 1/2 0/4 1/4 2/4 3/4 1/8; do
n=$(echo $s | tr / _)
LC_PLAN_BLOCK=$pb timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $s > $o/e${n}_pb$pb.json 2> /dev/null || exit 1
done
done
echo done
