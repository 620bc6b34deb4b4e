set -o pipefail
# r3final4: HEAD after the fuzz tests: GPU suite, smoke, default bench line
o=gpurun_out/r3final4; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_all.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $o/bench_default.json 2> $o/bench_default.err || exit 1
echo done
