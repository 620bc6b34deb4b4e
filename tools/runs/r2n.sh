set -o pipefail
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "not partitioned and not c4_full_size_grid and not c2_full" > $o/pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu --e2e-reps 0"
timeout -k 10 120 $B --steps 10 --warmup 3 > $o/c3.json 2> /dev/null || exit 1
LC_DEBUG=1 timeout -k 10 120 $B --steps 1 --warmup 1 > /dev/null 2> $o/c3_dbg.err || exit 1
timeout -k 10 120 $B --workload c1 --steps 20 --warmup 5 > $o/c1.json 2> /dev/null || exit 1
timeout -k 10 120 $B --workload c2 --steps 5 --warmup 2 > $o/c2.json 2> /dev/null || exit 1
timeout -k 10 200 $B --workload c4 --steps 1 --warmup 1 > $o/c4.json 2> /dev/null || exit 1
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 $B --steps 10 --warmup 3 --emulate $r/8 > $o/e$r.json 2> /dev/null || exit 1
done
echo done
