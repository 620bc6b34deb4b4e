set -o pipefail
# r3e: LC_PIPE bit 12 (a step after a hi return starts one super-layer after its predecessor)
# on the history teams: parity (the pipelined-step tests + full-size C2/C3 and random histories
# under LC_PIPE=8143), then A/B 4047 vs 8143 on C3, C1 and 8-way shares
o=gpurun_out/r3e; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "pipelined or low_slot" > $o/pytest_pipe.log 2>&1 || exit 1
LC_PIPE=8143 timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "c3_full or c2_full or c1_vs or random_small or kats or c3_subset or failure_configs or deterministic or shards_multiplexed or team" > $o/pytest_8143.log 2>&1 || exit 1
for i in 1 2; do
for pp in 4047 8143; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_${pp}_$i.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu --e2e-reps 0 > $o/c1_${pp}_$i.json 2> /dev/null || exit 1
done
done
for pp in 4047 8143; do
for r in 0 1 5; do
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}of8_$pp.json 2> /dev/null || exit 1
done
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_$pp.json 2> /dev/null || exit 1
done
LC_PIPE=8143 LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 0/8 > /dev/null 2> $o/e0of8_8143_debug.log || exit 1
echo done
