set -o pipefail
o=gpurun_out/r2tag; mkdir -p $o
LC_PIPE=463 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "tile_teams or c2_full or c3_subset or planner or c4_full_size_dense" > $o/pytest.log 2>&1 || exit 1
for pp in 207 463; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c4 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 3/8 > $o/e3_$pp.json 2> /dev/null || exit 1
done
LC_PIPE=463 LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c2 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_dbg.json 2> $o/c2_dbg.err || exit 1
echo done
