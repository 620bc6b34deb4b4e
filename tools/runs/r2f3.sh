set -o pipefail
o=gpurun_out/r2f3; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $o/bench_default.json 2> $o/bench_default.err || exit 1
timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 > $o/c1.json 2> $o/c1.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/c1_trace -o run -- python -u bench.py --workload c1 --no-cpu --e2e-reps 0 --steps 3 --warmup 1 > $o/c1_trace.log 2>&1 || exit 1
echo done
