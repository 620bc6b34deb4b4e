set -o pipefail
# r3i: which tile teams gain from rotation in a chain plan? every 8-way C3 share with and without
# LC_TEAM_ROT=32 (LC_DEBUG: team plan, per-tile phases, dense time), and rank 0 under forced tile
# sizes (LC_TILE_LBITS 14..17) with and without rotation
o=gpurun_out/r3i; mkdir -p $o
for r in 0 1 2 3 4 5 6 7; do
for rot in 0 32; do
LC_TEAM_ROT=$rot LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_r$rot.json 2> $o/e${r}_r$rot.log || exit 1
done
done
for lb in 15 16 17; do
for rot in 0 32; do
LC_TILE_LBITS=$lb LC_TEAM_ROT=$rot timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 0/8 > $o/e0_lb${lb}_r$rot.json 2> /dev/null || exit 1
done
done
echo done
