set -o pipefail
# r3ae: C2 on the HBM tables with fewer workgroups (cheaper grid barriers), and wide parity at 32
o=gpurun_out/r3ae; mkdir -p $o
LC_WIDE_GRID=32 timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q -k wide --timeout 120 --timeout-method thread > $o/pytest_wide32.log 2>&1 || exit 1
for g in 8 16 32 64 128; do
LC_WIDE_MINW=18 LC_WIDE_GRID=$g timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_wide_g$g.json 2> $o/c2_wide_g$g.log || exit 1
done
echo done
