set -o pipefail
# r3n: tile teams: credit tokens pre-polled a super-layer early (LC_PIPE bit 16) and a start gap
# of 3 after team-slot returns (bit 15): parity, then A/B on C2, C3 and the 8-way shares 0, 1;
# C3 LC_DEBUG at the default
o=gpurun_out/r3n; mkdir -p $o
LC_PIPE=118735 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "rotated or tile_teams or c3_subset or c2_full or random_small" > $o/pytest_new.log 2>&1 || exit 1
for rep in 1 2; do
for pp in 20431 85967 53199 118735; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 >> $o/c2_$pp.json 2> /dev/null || exit 1
for r in 0 1; do
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 >> $o/e${r}_$pp.json 2> /dev/null || exit 1
done
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_$pp.json 2> /dev/null || exit 1
done
done
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_debug.json 2> $o/c3_debug.log || exit 1
echo done
