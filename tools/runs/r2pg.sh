set -o pipefail
o=gpurun_out/r2pg; mkdir -p $o
for g in 32 64 128 256; do
LC_PART_GRID=$g timeout -k 10 300 python -u bench.py --workload c2 --partition --steps 1 --warmup 1 > $o/c2_g$g.json 2> $o/c2_g$g.err || exit 1
done
for g in 64 128; do
LC_PART_GRID=$g timeout -k 10 300 python -u bench.py --workload c4 --partition --steps 1 --warmup 0 > $o/c4_g$g.json 2> $o/c4_g$g.err || exit 1
done
echo done
