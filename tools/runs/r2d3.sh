set -o pipefail
o=gpurun_out/r2d3; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
bash tools/profile_round.sh r2i || exit 1
bash tools/profile_part.sh r2i
echo done
