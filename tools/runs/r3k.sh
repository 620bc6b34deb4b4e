set -o pipefail
# r3k: chain-plan rotation of 14-slot tiles with >= 4 team bits (auto); every 8-way share, rank 1
# under forced 14/15-slot tiles rotated; C2 LC_DEBUG (tile phases)
o=gpurun_out/r3k; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "rotated or tile_teams or c3_subset or shards_multiplexed" > $o/pytest_rot.log 2>&1 || exit 1
for r in 0 1 2 3 4 5 6 7; do
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}.json 2> /dev/null || exit 1
done
for lb in 14 15; do
LC_TILE_LBITS=$lb LC_TEAM_ROT=32 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 1/8 > $o/e1_lb${lb}_r32.json 2> /dev/null || exit 1
done
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c2 --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_debug.json 2> $o/c2_debug.log || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3.json 2> /dev/null || exit 1
echo done
