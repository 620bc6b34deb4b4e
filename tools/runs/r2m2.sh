set -o pipefail
o=gpurun_out/r2m2; mkdir -p $o
for g in 32 64 128 256; do
LC_PART_GRID=$g timeout -k 10 100 python -u bench.py --workload c2 --partition --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2p_g$g.json 2> $o/c2p_g$g.err || exit 1
done
echo done
