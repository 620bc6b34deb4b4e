set -o pipefail
o=gpurun_out/r2a3; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests/test_gpu.py -x -v --timeout 250 --timeout-method thread -k "dense or tile or c3 or c2_full or c4_full_size_dense or kats or random or failure or plan or determin" > $o/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3.json 2> /dev/null || exit 1
timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 > $o/c1.json 2> $o/c1.err || exit 1
timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2.json 2> /dev/null || exit 1
echo done
