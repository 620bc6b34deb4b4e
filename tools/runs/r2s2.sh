set -o pipefail
o=gpurun_out/r2s2; mkdir -p $o
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_def.json 2> /dev/null || exit 1
LC_TILE_LBITS=16 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_lb16.json 2> /dev/null || exit 1
LC_TILE_LBITS=15 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_lb15.json 2> /dev/null || exit 1
LC_TEAM_ROT_LB=17 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_rot17.json 2> /dev/null || exit 1
LC_BATCH_HIST=2000 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_chain.json 2> /dev/null || exit 1
echo done
