set -o pipefail
o=gpurun_out/r2l2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "partitioned and not c4 and not two_ranks" > $o/pytest.log 2>&1 || exit 1
timeout -k 10 100 python -u bench.py --workload c2 --partition --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2p.json 2> $o/c2p.err || exit 1
timeout -k 10 150 python -u bench.py --workload c4 --partition --capacity-log2 25 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > $o/c4p.json 2> $o/c4p.err || exit 1
echo done
