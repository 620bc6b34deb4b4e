#!/bin/bash
# Runs on the GPU box: axis-2 (partitioned frontier) profiles, written under gpurun_out/prof_<tag>/.
# The device-resident loop's rocprofv3 passes come last: rocprofv3 crashes in its own exit
# handler (SIGSEGV after "tool finalization") once it traced part_step_kernel's cooperative
# launches; the trace / counter files are complete by then.
# usage: tools/profile_part.sh <tag>
set -o pipefail
tag=$1
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python -u bench.py"
PP="python -u bench.py --workload c2 --partition --scale 0.3 --steps 1 --warmup 0"
# host-driven level protocol (part_expand / part_absorb, as world > 1 runs)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/partp_trace -o run -- $PP --level-protocol \
  > $out/partp_trace.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum \
  TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum --output-format csv -d $out/partp_pmc_atomic -o run -- $PP --level-protocol \
  > $out/partp_pmc.log 2>&1 || exit 1
timeout -k 10 400 $B --workload c4 --partition --steps 1 --warmup 0 > $out/c4_partition_bench.json 2> $out/c4_partition_bench.err || exit 1
timeout -k 10 400 $B --workload c2 --partition --steps 2 --warmup 1 > $out/c2_partition_bench.json 2> $out/c2_partition_bench.err || exit 1
timeout -k 10 200 $B --workload c4 --steps 1 --warmup 1 --no-cpu > $out/c4_bench.json 2> $out/c4_bench.err || exit 1
# device-resident loop (lc_part_run, flow kernel by default): kernel trace, then the atomic
# counters (both may end in rocprofv3's exit-handler crash after the files are written)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/part_trace -o run -- $PP \
  > $out/part_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum \
  TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum --output-format csv -d $out/part_pmc_atomic -o run -- $PP > $out/part_pmc.log 2>&1
echo done
