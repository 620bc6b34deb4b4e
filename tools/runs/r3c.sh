set -o pipefail
# r3c: full GPU suite (persistent encoder pool, streams built inside the encoder), default
# bench (C3) and C1/C2 lines with the lc_check phase split, C2 PMC passes at the final kernel,
# then the rocprofv3 exit experiment on a cooperative grid-kernel run (last: it may fault)
o=gpurun_out/r3c; mkdir -p $o
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
LC_PHASES=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $o/c3.json 2> $o/c3.err || exit 1
LC_PHASES=1 timeout -k 10 200 python -u bench.py --workload c1 --steps 50 --warmup 10 --e2e-reps 9 > $o/c1.json 2> $o/c1.err || exit 1
LC_PIPE=4047 timeout -k 10 200 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu --e2e-reps 9 > $o/c1_fix.json 2> $o/c1_fix.err || exit 1
LC_PIPE=4047 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_fix.json 2> $o/c3_fix.err || exit 1
for rot in 1 2 3; do
LC_TEAM_ROT=$rot timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 0/8 > $o/e0of8_rot$rot.json 2> /dev/null || exit 1
done
for lb in 13 15; do
LC_TILE_LBITS=$lb timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 0/8 > $o/e0of8_lb$lb.json 2> /dev/null || exit 1
done
timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 > $o/c2.json 2> $o/c2.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="python -u bench.py --workload c2 --no-cpu --e2e-reps 0 --steps 1 --warmup 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/c2_trace -o run -- python -u bench.py --workload c2 --no-cpu --e2e-reps 0 --steps 3 --warmup 1 > $o/c2_trace.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/c2_pmc_fetch -o run -- $P > $o/pmc.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/c2_pmc_write -o run -- $P >> $o/pmc.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $o/c2_pmc_sq -o run -- $P >> $o/pmc.log 2>&1 || exit 1
LC_PATH=grid LC_MAPS_DUMP=$PWD/$o/grid_maps.txt timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/grid_trace -o run -- python -u bench.py --workload c1 --no-cpu --e2e-reps 0 --steps 2 --warmup 1 > $o/grid_trace.log 2>&1
echo "grid trace rc=$?" >> $o/grid_trace.log
echo done
