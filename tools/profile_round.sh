#!/bin/bash
# Runs on the GPU box: bench line + rocprofv3 kernel trace/stats + PMC passes (HBM traffic,
# then vector/scalar/LDS instruction counts), each pass a run of its own.
# usage: tools/profile_round.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python -u bench.py "$@" --no-cpu --steps 2 --warmup 1 > $out/trace.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- \
  python -u bench.py "$@" --no-cpu --steps 1 --warmup 0 > $out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- \
  python -u bench.py "$@" --no-cpu --steps 1 --warmup 0 > $out/pmc_write.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES \
  SQ_WAVE_CYCLES --output-format csv -d $out/pmc_sq -o run -- \
  python -u bench.py "$@" --no-cpu --steps 1 --warmup 0 > $out/pmc_sq.log 2>&1 || exit 1
echo done
