set -o pipefail
o=gpurun_out/r2r; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "two_ranks or failure or checker_api or kats or errors or c3_full" > $o/pytest.log 2>&1 || exit 1
LC_PHASES=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 5 > $o/c3.json 2> $o/c3.err || exit 1
echo done
