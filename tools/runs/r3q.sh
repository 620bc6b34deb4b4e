set -o pipefail
# r3q: closure tables in HBM (wide.hip): parity tests, the crash ramp past width 24 on them,
# then the planner sweep of r3p (LC_PLAN_ROT=1 around LC_PLAN_KB 0.6)
o=gpurun_out/r3q; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "wide" > $o/pytest_wide.log 2>&1 || exit 1
timeout -k 10 700 python -u tools/crash_ramp.py --ops 2000 --crashed 10,12,13,14,16 --no-cpu --gpu-timeout 150 > $o/ramp_wide.jsonl 2> $o/ramp_wide.log || exit 1
LC_DEBUG=1 timeout -k 10 200 python -u tools/crash_ramp.py --ops 2000 --crashed 13 --no-cpu --gpu-timeout 150 > /dev/null 2> $o/ramp_k13_debug.log || exit 1
bash tools/runs/r3p.sh || exit 1
echo done
