set -o pipefail
o=gpurun_out/r2s; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "partitioned" > $o/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --partition --workload c2 --steps 2 --warmup 1 > $o/c2p.json 2> $o/c2p.err || exit 1
timeout -k 10 300 python -u bench.py --partition --workload c4 --steps 1 --warmup 0 > $o/c4p.json 2> $o/c4p.err || exit 1
echo done
