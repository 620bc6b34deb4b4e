set -o pipefail
o=gpurun_out/r2tw2; mkdir -p $o
LC_TILE_WIDE=19:14 LC_MID_MAXW=12 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/4 > $o/a.json 2> /dev/null || exit 1
LC_TILE_WIDE=19:14 LC_PIPE=335 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/4 > $o/b.json 2> /dev/null || exit 1
LC_MID_MAXW=12 LC_PLAN_K=1.0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/4 > $o/c.json 2> /dev/null || exit 1
LC_PIPE=335 LC_PLAN_K=1.0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/4 > $o/d.json 2> /dev/null || exit 1
echo done
