set -o pipefail
o=gpurun_out/r2e3; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "1999" > $o/pytest.log 2>&1 || exit 1
for pp in 975 1999; do
LC_PIPE=$pp timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu --e2e-reps 0 > $o/c1_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/8 > $o/e2_$pp.json 2> /dev/null || exit 1
done
echo done
