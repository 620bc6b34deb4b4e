set -o pipefail
o=gpurun_out/r2j; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "not c4 and not partitioned and not c2_full" > $o/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3.json 2> $o/c3.err || exit 1
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c3_dbg.err || exit 1
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e$r.json 2> /dev/null || exit 1
done
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 2/8 > /dev/null 2> $o/e2_dbg.err || exit 1
timeout -k 10 120 python -u bench.py --workload c1 --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c1.json 2> /dev/null || exit 1
timeout -k 10 120 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2.json 2> /dev/null || exit 1
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --workload c2 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c2_dbg.err || exit 1
echo done
