set -o pipefail
# r3l: LC_PIPE bit 14 (XCD-compact workgroup roles): parity subset, A/B on C2 / C3 / shares 0, 1;
# the C4 crash ramp (tools/crash_ramp.py: 2,000-op histories, 16 clients, K crashed ops);
# C2 under partial rotations and tile sizes
o=gpurun_out/r3l; mkdir -p $o
LC_PIPE=20431 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "rotated or tile_teams or c3_subset or c2_full or kats or random_small" > $o/pytest_xcd.log 2>&1 || exit 1
for pp in 4047 20431 4047 20431; do
for r in 0 1; do
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_$pp.json 2> /dev/null || exit 1
done
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_$pp.json 2> /dev/null || exit 1
done
timeout -k 10 900 python -u tools/crash_ramp.py --ops 2000 --crashed 0,2,4,5,6,7,8,9,10,12,14,16 --cpu-timeout 60 --gpu-timeout 100 --part > $o/ramp.jsonl 2> $o/ramp.log || exit 1
for lb in 13 14 15; do
for rot in 1 2 3; do
LC_TILE_LBITS=$lb LC_TEAM_ROT=$rot timeout -k 10 120 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_lb${lb}_r$rot.json 2> /dev/null || exit 1
done
done
echo done
