set -o pipefail
# r3u: HBM tables up to 31 live slots: wide parity tests (a width-31 case added), ramp K = 16, 17
o=gpurun_out/r3u; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "wide" > $o/pytest_wide.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/crash_ramp.py --ops 2000 --crashed 16,17 --no-cpu --gpu-timeout 150 > $o/ramp.jsonl 2> $o/ramp.log || exit 1
echo done
