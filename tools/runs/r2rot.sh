set -o pipefail
o=gpurun_out/r2rot; mkdir -p $o
for r in 0 2 4 7; do
LC_TEAM_ROT=$r timeout -k 10 120 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > $o/c4_r$r.json 2> $o/c4_r$r.err || exit 1
done
for r in 0 1 2 3 5; do
LC_TEAM_ROT=$r timeout -k 10 120 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_r$r.json 2> $o/c2_r$r.err || exit 1
done
for r in 1 2 3; do
LC_TEAM_ROT=$r timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_r$r.json 2> $o/c3_r$r.err || exit 1
done
LC_TEAM_ROT=3 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "tile_teams or c2_full or c3_subset or planner" > $o/pytest_rot3.log 2>&1 || exit 1
echo done
