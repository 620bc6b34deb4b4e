#!/bin/bash
# Runs on the GPU box: the round's bench lines, rocprofv3 kernel trace/stats, and PMC passes
# (HBM traffic, instruction counts, and the partitioned kernels' atomics), each pass a run of
# its own, written under gpurun_out/prof_<tag>/.
# usage: tools/profile_round.sh <tag>
set -o pipefail
tag=$1
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python -u bench.py"
# bench lines (C3 default first, as the driver runs it)
timeout -k 10 300 $B --steps 20 --warmup 5 > $out/c3_bench.json 2> $out/c3_bench.err || exit 1
timeout -k 10 200 $B --workload c1 --steps 50 --warmup 10 > $out/c1_bench.json 2> $out/c1_bench.err || exit 1
timeout -k 10 200 $B --workload c2 --steps 10 --warmup 2 > $out/c2_bench.json 2> $out/c2_bench.err || exit 1
timeout -k 10 200 $B --workload c5 --steps 20 --warmup 5 > $out/c5_bench.json 2> $out/c5_bench.err || exit 1
timeout -k 10 300 $B --workload c4 --steps 3 --warmup 1 > $out/c4_bench.json 2> $out/c4_bench.err || exit 1
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 $B --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $out/c3_emulate_${r}of8.json 2> /dev/null || exit 1
done
# kernel traces + stats
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c3_trace -o run -- \
  python -u bench.py --no-cpu --e2e-reps 0 --steps 3 --warmup 1 > $out/c3_trace.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c2_trace -o run -- \
  python -u bench.py --workload c2 --no-cpu --e2e-reps 0 --steps 3 --warmup 1 > $out/c2_trace.log 2>&1 || exit 1
# PMC passes on C3 (one launch each)
P="python -u bench.py --no-cpu --e2e-reps 0 --steps 1 --warmup 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/c3_pmc_fetch -o run -- $P > $out/pmc.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/c3_pmc_write -o run -- $P >> $out/pmc.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d $out/c3_pmc_sq -o run -- $P >> $out/pmc.log 2>&1 || exit 1
# C2 PMC: SQ (one width-18 history on a planned team)
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d $out/c2_pmc_sq -o run -- python -u bench.py --workload c2 --no-cpu --e2e-reps 0 --steps 1 \
  --warmup 0 >> $out/pmc.log 2>&1 || exit 1
# partitioned frontier: tools/profile_part.sh (its own call: rocprofv3 segfaults at exit after
# tracing the cooperative part_step_kernel, once the trace is written)
# the HBM-table kernel (crash ramp K = 16, width 30), last: it is a cooperative launch, and
# rocprofv3 runs over cooperative kernels fault in the HIP runtime's exit handler after the
# profile is written: one pass, the script's last GPU command, its exit status recorded
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/wide_trace -o run -- python -u tools/wide_once.py 16 > $out/wide_trace.log 2>&1; echo "wide trace exit $?" >> $out/pmc.log
echo done
