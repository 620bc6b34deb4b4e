set -o pipefail
o=gpurun_out/r2x2; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 250 --timeout-method thread -k "rotated or c4_full_size_dense or tile or c3_full" > $o/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3.json 2> /dev/null || exit 1
timeout -k 10 200 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4.json 2> /dev/null || exit 1
timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2.json 2> /dev/null || exit 1
for r in 0 3 5; do
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e$r.json 2> /dev/null || exit 1
done
echo done
