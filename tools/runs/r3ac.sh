set -o pipefail
# r3ac: one WAVE history per workgroup (LC_PIPE bit 18) with the grid sized for it: parity, then C1/C2/C3 A/B
o=gpurun_out/r3ac; mkdir -p $o
LC_PIPE=479183 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > $o/pytest_spread.log 2>&1 || exit 1
for w in c1 c2 c3; do
for pp in 217039 479183 217039 479183; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 2 --no-cpu --e2e-reps 0 >> $o/${w}_$pp.json 2>> $o/${w}_$pp.log || exit 1
done
done
echo done
