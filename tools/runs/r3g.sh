set -o pipefail
# r3g: LC_PIPE bit 13 (global popcount layers for tile teams): parity first (the new tile-team
# tests, the pipelined-step tests, full-size C2/C3/C4-scale suites under LC_PIPE=12239), then
# A/B on the chains it targets: the 8-way C3 shares, C2, C3 at one GPU, forced rotation
o=gpurun_out/r3g; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "global_layers or pipelined_steps" > $o/pytest_glay.log 2>&1 || exit 1
LC_PIPE=12239 timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "c3_full or c2_full or c1_vs or random_small or kats or c3_subset or failure_configs or deterministic or shards_multiplexed or team" > $o/pytest_12239.log 2>&1 || exit 1
for pp in 4047 12239; do
for r in 0 1 5; do
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}of8_$pp.json 2> /dev/null || exit 1
LC_TEAM_ROT=32 LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}of8_${pp}_rot.json 2> /dev/null || exit 1
done
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_$pp.json 2> /dev/null || exit 1
LC_TEAM_ROT=32 LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_${pp}_rot.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_$pp.json 2> /dev/null || exit 1
done
for pp in 4047 12239; do
LC_PIPE=$pp LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 0/8 > /dev/null 2> $o/e0of8_${pp}_debug.log || exit 1
LC_TEAM_ROT=32 LC_PIPE=$pp LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 0/8 > /dev/null 2> $o/e0of8_${pp}_rot_debug.log || exit 1
done
echo done
