set -o pipefail
# r3o: the team model aware of rotated teams (LC_PLAN_ROT=1: every step spread over the tiles
# and paying the exchange) x the batch plan's VALU factor LC_PLAN_KB, on C3; the 8-way shares
# under LC_PLAN_ROT=1; defaults otherwise (LC_PIPE unset: 85967)
o=gpurun_out/r3o; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "c3_full or tile_teams_rotated or pipelined_steps" > $o/pytest.log 2>&1 || exit 1
for rep in 1 2; do
for pr in 0 1; do
for kb in 0.45 0.6 0.8; do
LC_PLAN_ROT=$pr LC_PLAN_KB=$kb timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_r${pr}_k$kb.json 2> /dev/null || exit 1
done
done
done
for r in 0 1 2 3 4 5 6 7; do
for pr in 0 1; do
LC_PLAN_ROT=$pr timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_r$pr.json 2> /dev/null || exit 1
done
done
LC_PLAN_ROT=1 LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_rot_debug.json 2> $o/c3_rot_debug.log || exit 1
echo done
