set -o pipefail
# r3j: LC_PIPE bit 14 (skip the in-word closure of words without configs): parity subset, then
# A/B {4047, 20431} on C3, C2 and the 8-way shares 0, 1, 4 (LC_TEAM_ROT auto)
o=gpurun_out/r3j; mkdir -p $o
LC_PIPE=20431 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "c3_full or c2_full or random_small or c3_subset or failure_configs or tile_teams or kats" > $o/pytest_zskip.log 2>&1 || exit 1
for pp in 4047 20431 4047 20431; do
for r in 0 1 4; do
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_$pp.json 2> /dev/null || exit 1
done
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_$pp.json 2> /dev/null || exit 1
done
echo done
