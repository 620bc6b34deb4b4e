set -o pipefail
# r3x: HEAD check as the driver runs it: the whole GPU suite, smoke(), the default bench line
o=${O:-gpurun_out/r3x}; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest_all.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $o/bench_default.json 2> $o/bench_default.err || exit 1
echo done
