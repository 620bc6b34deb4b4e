set -o pipefail
# r3aq: the fuzz parity tests at large sizes (4000 register + 800 counter; 1200 wide)
o=gpurun_out/r3aq; mkdir -p $o
LC_FUZZ_N=4000 timeout -k 10 800 python -u -m pytest tests/test_gpu.py -x -v -k "fuzz_register" --timeout 790 --timeout-method thread > $o/fuzz4000.log 2>&1 || exit 1
LC_FUZZ_WIDE_N=1200 timeout -k 10 800 python -u -m pytest tests/test_gpu.py -x -v -k fuzz_wide --timeout 790 --timeout-method thread > $o/fuzzw1200.log 2>&1 || exit 1
echo done
