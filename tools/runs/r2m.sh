set -o pipefail
o=gpurun_out/r2m; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "c4 or dense or kats or planner" > $o/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4.json 2> $o/c4.err || exit 1
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c4_dbg.err || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3.json 2> /dev/null || exit 1
echo done
