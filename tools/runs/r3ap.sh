set -o pipefail
# r3ap: the wide fuzz parity test at its default size and at 300 histories
o=gpurun_out/r3ap; mkdir -p $o
timeout -k 10 280 python -u -m pytest tests/test_gpu.py -x -v -k fuzz_wide --timeout 270 --timeout-method thread > $o/fuzzw60.log 2>&1 || exit 1
LC_FUZZ_WIDE_N=300 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v -k fuzz_wide --timeout 590 --timeout-method thread > $o/fuzzw300.log 2>&1 || exit 1
echo done
