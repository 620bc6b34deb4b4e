set -o pipefail
# r3z: tagged tile teams stage the X words of team-slot returns a super-layer early (LC_PIPE bit
# 18): parity, then A/B {217039 (default), 479183} on C2, C3, C4 and the 8-way shares 0, 1
o=gpurun_out/r3z; mkdir -p $o
LC_PIPE=479183 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "rotated or tile_teams or c3_subset or c2_full or c4_full_size_dense or global_layers" > $o/pytest_xpre.log 2>&1 || exit 1
for rep in 1 2; do
for pp in 217039 479183; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 >> $o/c2_$pp.json 2> /dev/null || exit 1
for r in 0 1; do
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 >> $o/e${r}_$pp.json 2> /dev/null || exit 1
done
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_$pp.json 2> /dev/null || exit 1
done
done
for pp in 217039 479183; do
LC_PIPE=$pp timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --e2e-reps 0 >> $o/c4_$pp.json 2> /dev/null || exit 1
done
LC_PIPE=479183 LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c2 --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c2_xpre_debug.log || exit 1
echo done
