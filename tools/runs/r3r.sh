set -o pipefail
# r3r: the whole GPU suite at HEAD; C4 bench line; a kernel trace of the HBM-table kernel on the
# crash ramp's width-30 history (K = 16)
o=gpurun_out/r3r; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest_all.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 > $o/c4_bench.json 2> $o/c4_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/wide_trace -o run -- python -u tools/wide_once.py 16 > $o/wide_trace.log 2>&1; echo "wide trace exit $?" > $o/wide_trace.status
echo done
