set -o pipefail
o=gpurun_out/r2e; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "tile or planner or c2_full" > $o/pytest.log 2>&1 || exit 1
for lb in 16 15 14 13; do
  LC_TILE_LBITS=$lb timeout -k 10 120 python -u bench.py --workload c2 --steps 3 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_l$lb.json 2> /dev/null || exit 1
done
for lb in 16 15 14; do
  for r in 1 2; do
    LC_TILE_LBITS=$lb timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_l$lb.json 2> /dev/null || exit 1
  done
done
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 1/8 > /dev/null 2> $o/e1_dbg.err || exit 1
LC_DEBUG=1 LC_TILE_LBITS=14 timeout -k 10 120 python -u bench.py --workload c2 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c2_l14_dbg.err || exit 1
echo done
