set -o pipefail
# r3ad: C2 (one width-18 history) on the HBM tables' whole-grid pipelined schedule vs the tile team
o=gpurun_out/r3ad; mkdir -p $o
timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_team.json 2> $o/c2_team.log || exit 1
LC_WIDE_MINW=18 timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_wide.json 2> $o/c2_wide.log || exit 1
LC_WIDE_MINW=18 LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c2 --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_wide_dbg.json 2> $o/c2_wide_dbg.log || exit 1
echo done
