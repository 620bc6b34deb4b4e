set -o pipefail
mkdir -p gpurun_out/r2a
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export LC_PHASES=1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1 || exit 1
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu --e2e-reps 1 --emulate $r/8 > gpurun_out/r2a/emu$r.json 2>> gpurun_out/r2a/emu.err || exit 1
done
rocprofv3 --list-avail > gpurun_out/r2a/avail.txt 2>&1 || true
echo done
