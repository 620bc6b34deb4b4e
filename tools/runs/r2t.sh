set -o pipefail
o=gpurun_out/r2t; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "pipelined_steps or low_slot" > $o/pytest.log 2>&1 || exit 1
LC_PIPE=207 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "kats or c3 or random or dense_tables or planner or c1" > $o/pytest207.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_79.json 2> $o/c3_79.err || exit 1
LC_PIPE=207 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_207.json 2> $o/c3_207.err || exit 1
LC_PIPE=207 LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_207_dbg.json 2> $o/c3_207_dbg.err || exit 1
echo done
