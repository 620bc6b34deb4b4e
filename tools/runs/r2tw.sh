set -o pipefail
o=gpurun_out/r2tw; mkdir -p $o
for tw in 19:14 19:13 20:14 99:17; do
n=$(echo $tw | tr : _)
LC_TILE_WIDE=$tw timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/4 > $o/s2_4_$n.json 2> /dev/null || exit 1
done
LC_DEBUG=1 LC_TILE_WIDE=19:14 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 2/4 > $o/dbg.json 2> $o/dbg.err || exit 1
echo done
