set -o pipefail
o=gpurun_out/r2r2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "pipelined or low_slot or c1 or kats or random" > $o/pytest.log 2>&1 || exit 1
for ww in 16 4 1; do
LC_WAVE_WG=$ww timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu --e2e-reps 0 > $o/c1_w$ww.json 2> /dev/null || exit 1
done
timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 > $o/c1.json 2> $o/c1.err || exit 1
for r in 0 3 5; do
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e$r.json 2> /dev/null || exit 1
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3.json 2> $o/c3.err || exit 1
echo done
