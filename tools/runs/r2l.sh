set -o pipefail
o=gpurun_out/r2l; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
LC_PHASES=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $o/c3.json 2> $o/c3.err || exit 1
echo done
