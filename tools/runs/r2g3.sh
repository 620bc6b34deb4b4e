set -o pipefail
o=gpurun_out/r2g3; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "pipelined_steps and 1999 or low_slot and 1999 or tile_teams_rotated" > $o/pytest_dense.log 2>&1 || true
for pp in 1999 4047; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/8 > $o/e2_$pp.json 2> /dev/null || exit 1
done
LC_PIPE=4047 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "pipelined_steps or low_slot or tile_teams or c3_subset or c2_full" > $o/pytest_sparse.log 2>&1 || exit 1
echo done
