set -o pipefail
# r3h: tile-team step ring 16 -> 32 (global layers lengthen a step's span by T); parity of the
# leader model and the tile-team variants, then A/B {4047, 12239} x {unrotated, LC_TEAM_ROT=32}
o=gpurun_out/r3h; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "leader or global_layers or rotated or pipelined_steps or tile_teams" > $o/pytest_a.log 2>&1 || exit 1
LC_PIPE=12239 LC_TEAM_ROT=32 timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "c3_full or c2_full or random_small or c3_subset or failure_configs or shards_multiplexed" > $o/pytest_glay_rot.log 2>&1 || exit 1
for pp in 4047 12239; do
for rot in 0 32; do
for r in 0 1 5; do
LC_TEAM_ROT=$rot LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}of8_${pp}_r$rot.json 2> /dev/null || exit 1
done
LC_TEAM_ROT=$rot LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_${pp}_r$rot.json 2> /dev/null || exit 1
done
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_$pp.json 2> /dev/null || exit 1
done
LC_TEAM_ROT=32 LC_PIPE=12239 LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 0/8 > /dev/null 2> $o/e0of8_12239_rot_debug.log || exit 1
echo done
