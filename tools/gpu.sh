#!/bin/bash
# Host-side wrapper: re-submit only when gpurun reports "no box/slot" or a transient
# infrastructure event (exit 3: nothing ran, nothing charged). Any other outcome returns.
# usage: tools/gpu.sh <timeout_s> '<command>'
to=$1; shift
for i in $(seq 1 ${GPU_RETRIES:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpu.sh] transient (exit 3), retry $i in 60s" >&2
  sleep 60
done
exit 3
