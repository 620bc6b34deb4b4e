set -o pipefail
o=gpurun_out/r2i3; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $o/c3.json 2> $o/c3.err || exit 1
timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 > $o/c2.json 2> $o/c2.err || exit 1
timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 > $o/c1.json 2> $o/c1.err || exit 1
timeout -k 10 200 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu > $o/c4.json 2> $o/c4.err || exit 1
for r in 0 1 2 3 4 5 6 7; do
timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/c3_emulate_${r}of8.json 2> /dev/null || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/c3_trace -o run -- python -u bench.py --no-cpu --e2e-reps 0 --steps 3 --warmup 1 > $o/c3_trace.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/c2_trace -o run -- python -u bench.py --workload c2 --no-cpu --e2e-reps 0 --steps 3 --warmup 1 > $o/c2_trace.log 2>&1 || exit 1
P="python -u bench.py --no-cpu --e2e-reps 0 --steps 1 --warmup 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/c3_pmc_fetch -o run -- $P > $o/pmc.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/c3_pmc_write -o run -- $P >> $o/pmc.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $o/c3_pmc_sq -o run -- $P >> $o/pmc.log 2>&1 || exit 1
echo done
