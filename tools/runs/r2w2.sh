set -o pipefail
o=gpurun_out/r2w2; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 250 --timeout-method thread -k "dense or c2_full or c4 or c3_full or kats or random or partitioned_world1" > $o/pytest.log 2>&1 || exit 1
for sp in lff smart; do
LC_SLOTS=$sp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_$sp.json 2> /dev/null || exit 1
LC_SLOTS=$sp timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_$sp.json 2> /dev/null || exit 1
LC_SLOTS=$sp timeout -k 10 200 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4_$sp.json 2> /dev/null || exit 1
LC_SLOTS=$sp timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu --e2e-reps 0 > $o/c1_$sp.json 2> /dev/null || exit 1
for r in 0 3 5; do
LC_SLOTS=$sp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_$sp.json 2> /dev/null || exit 1
done
done
echo done
