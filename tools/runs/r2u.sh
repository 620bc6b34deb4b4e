set -o pipefail
o=gpurun_out/r2u; mkdir -p $o
LC_PIPE=207 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "kats or c3 or random or dense or planner or c1 or c2_full" > $o/pytest207.log 2>&1 || exit 1
for k in 1.3 1.6 2.0; do
LC_PLAN_K=$k LC_PIPE=207 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_207_k$k.json 2> $o/c3_207_k$k.err || exit 1
done
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_79.json 2> $o/c3_79.err || exit 1
LC_PIPE=207 LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_207_dbg.json 2> $o/c3_207_dbg.err || exit 1
echo done
