set -o pipefail
o=gpurun_out/r2pmc; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in c2 c4; do
P="python -u bench.py --workload $w --no-cpu --e2e-reps 0 --steps 1 --warmup 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/${w}_pmc_fetch -o run -- $P > $o/${w}_pmc.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/${w}_pmc_write -o run -- $P >> $o/${w}_pmc.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d $o/${w}_pmc_sq -o run -- $P >> $o/${w}_pmc.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${w}_trace -o run -- $P > $o/${w}_trace.log 2>&1 || exit 1
done
echo done
