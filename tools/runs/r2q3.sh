set -o pipefail
o=gpurun_out/r2q3; mkdir -p $o
for lb in 12 13 14 15; do
LC_TILE_LBITS=$lb timeout -k 10 120 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_lb$lb.json 2> /dev/null || exit 1
done
echo done
