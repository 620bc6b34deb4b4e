set -o pipefail
# r3t: the pipelined HBM-table kernel (LC_WIDE_PIPE=1, default): wide parity tests (both forms),
# the crash ramp's wide legs with and without pipelining
o=gpurun_out/r3t; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "wide" > $o/pytest_wide.log 2>&1 || exit 1
for pp in 1 0; do
LC_WIDE_PIPE=$pp timeout -k 10 400 python -u tools/crash_ramp.py --ops 2000 --crashed 12,13,14,16 --no-cpu --gpu-timeout 150 > $o/ramp_pipe$pp.jsonl 2> $o/ramp_pipe$pp.log || exit 1
done
echo done
