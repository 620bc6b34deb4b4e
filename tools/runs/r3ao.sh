set -o pipefail
# r3ao: the fuzz parity test at its default size and at 2000 register histories (+400 counters)
o=gpurun_out/r3ao; mkdir -p $o
timeout -k 10 280 python -u -m pytest tests/test_gpu.py -x -v -k fuzz --timeout 270 --timeout-method thread > $o/fuzz200.log 2>&1 || exit 1
LC_FUZZ_N=2000 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v -k fuzz --timeout 590 --timeout-method thread > $o/fuzz2000.log 2>&1 || exit 1
echo done
