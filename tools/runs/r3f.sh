set -o pipefail
# r3f: lc_part_check per-level cost (C2 over 1/2/4 in-process ranks on one GPU), the cost split's
# 2- and 4-way shares, and the round's C3 profile set: default bench line, kernel trace + stats,
# PMC passes (FETCH / WRITE / SQ) of one launch
o=gpurun_out/r3f; mkdir -p $o
for n in 1 2 4; do
timeout -k 10 300 python -u bench.py --workload c2 --partition --in-process $n --steps 2 --warmup 1 > $o/c2_inproc_$n.json 2> $o/c2_inproc_$n.err || exit 1
done
for r in 0 1; do
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/2 > $o/e${r}of2.json 2> /dev/null || exit 1
done
for r in 0 1 2 3; do
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/4 > $o/e${r}of4.json 2> /dev/null || exit 1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $o/c3_bench.json 2> $o/c3_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="python -u bench.py --no-cpu --e2e-reps 0 --steps 1 --warmup 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/c3_trace -o run -- python -u bench.py --no-cpu --e2e-reps 0 --steps 5 --warmup 1 > $o/c3_trace.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/c3_pmc_fetch -o run -- $P > $o/pmc.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/c3_pmc_write -o run -- $P >> $o/pmc.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $o/c3_pmc_sq -o run -- $P >> $o/pmc.log 2>&1 || exit 1
echo done
