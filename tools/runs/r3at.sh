set -o pipefail
# r3at: HEAD (chain-rotation knob added, defaults unchanged): team/planner GPU tests, C2/C3 full size, smoke
o=gpurun_out/r3at; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q -k "team or planner or c2_full or c3 or fuzz" --timeout 300 --timeout-method thread > $o/pytest_sub.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
echo done
