set -o pipefail
# r3af: C2 with tiles below the planner's 13-slot floor (LC_TILE_LBITS 13/12/11/10: 32..256 workgroups)
o=gpurun_out/r3af; mkdir -p $o
for lb in 13 12 11 10; do
LC_TILE_LBITS=$lb timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_lb$lb.json 2> $o/c2_lb$lb.log || exit 1
done
LC_TILE_LBITS=12 LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c2 --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_lb12_dbg.json 2> $o/c2_lb12_dbg.log || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q -k wide_tables_vs --timeout 120 --timeout-method thread > $o/pytest_wide.log 2>&1 || exit 1
echo done
