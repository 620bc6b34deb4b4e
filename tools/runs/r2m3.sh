set -o pipefail
o=gpurun_out/r2m3; mkdir -p $o
for lb in 13 14 15 16; do
LC_TILE_LBITS=$lb timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/8 > $o/e2_lb$lb.json 2> /dev/null || exit 1
done
for rot in 0 3; do
LC_TEAM_ROT=$rot timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/8 > $o/e2_rot$rot.json 2> /dev/null || exit 1
done
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/8 > $o/e2_def.json 2> /dev/null || exit 1
echo done
