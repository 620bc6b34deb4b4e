set -o pipefail
o=gpurun_out/r2v2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 250 --timeout-method thread -k "c3_full_size" > $o/pytest.log 2>&1 || exit 1
echo done
