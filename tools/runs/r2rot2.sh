set -o pipefail
o=gpurun_out/r2rot2; mkdir -p $o
for lb in 14 15 16 17; do
LC_TILE_WIDE=19:$lb LC_TEAM_ROT=9 timeout -k 10 120 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > $o/c4_lb${lb}_rot.json 2> $o/c4_lb${lb}_rot.err || exit 1
done
for lb in 13 14 15 16 17; do
for r in 0 9; do
LC_TILE_WIDE=18:$lb LC_TEAM_ROT=$r timeout -k 10 120 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_lb${lb}_r$r.json 2> $o/c2_lb${lb}_r$r.err || exit 1
done
done
echo done
