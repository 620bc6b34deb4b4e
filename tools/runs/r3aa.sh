set -o pipefail
# r3aa: C1's WAVE (REG) histories one per workgroup (LC_PIPE bit 18) vs 16 per workgroup: parity,
# then A/B on C1 (kernel and end to end), 3 alternating passes
o=gpurun_out/r3aa; mkdir -p $o
LC_PIPE=479183 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "c1 or random_small or kats" > $o/pytest_spread.log 2>&1 || exit 1
for rep in 1 2 3; do
for pp in 217039 479183; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu >> $o/c1_$pp.json 2> /dev/null || exit 1
done
done
echo done
