set -o pipefail
o=gpurun_out/r2h; mkdir -p $o
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $o/c3.json 2> $o/c3.err || exit 1
timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu > $o/c2.json 2> $o/c2.err || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
echo done
