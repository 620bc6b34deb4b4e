set -o pipefail
o=gpurun_out/r2z2; mkdir -p $o
for g in 64 128 192 256; do
LC_PART_GRID=$g timeout -k 10 100 python -u bench.py --workload c2 --partition --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2p_g$g.json 2> /dev/null || exit 1
done
for g in 128 256; do
LC_PART_GRID=$g timeout -k 10 150 python -u bench.py --workload c4 --partition --capacity-log2 25 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > $o/c4p_g$g.json 2> /dev/null || exit 1
done
echo done
