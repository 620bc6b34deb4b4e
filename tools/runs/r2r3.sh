set -o pipefail
o=gpurun_out/r2r3; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "tile_teams or c2_full or planner" > $o/pytest.log 2>&1 || exit 1
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --workload c2 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c2_dbg.err || exit 1
timeout -k 10 120 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2.json 2> /dev/null || exit 1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3.json 2> /dev/null || exit 1
for s in 1/2 2/4 2/8; do
n=$(echo $s | tr / _)
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $s > $o/e$n.json 2> /dev/null || exit 1
done
echo done
