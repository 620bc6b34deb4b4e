set -o pipefail
o=gpurun_out/r2j; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "dense or full or c2 or c4" > $o/pytest.log 2>&1 || exit 1
for pp in 463 975; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_$pp.json 2> $o/c3_$pp.err || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_$pp.json 2> $o/c2_$pp.err || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4_$pp.json 2> $o/c4_$pp.err || exit 1
for r in 0 3 5; do
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_$pp.json 2> /dev/null || exit 1
done
done
echo done
