set -o pipefail
o=gpurun_out/r2u3; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $o/bench.json 2> $o/bench.err || exit 1
echo done
