set -o pipefail
# r3m: the whole GPU suite at the new defaults (LC_PIPE 20431: XCD-compact roles; chain-plan
# rotation of 14-slot teams), then the crash ramp's GPU legs past the dense limit (grid kernel)
o=gpurun_out/r3m; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest_all.log 2>&1 || exit 1
timeout -k 10 700 python -u tools/crash_ramp.py --ops 2000 --crashed 10,12,13,14 --no-cpu --gpu-timeout 300 > $o/ramp_gpu.jsonl 2> $o/ramp_gpu.log || exit 1
echo done
