#!/bin/bash
# One parameterised GPU-box runner (replaces round 2/3's one-off tools/runs/*.sh).
# Every step writes under gpurun_out/<tag>/, runs under its own time limit, and the script stops
# at the first failing step (no retries, nothing started on the GPU after a fault or timeout).
#
# usage: tools/run.sh <tag> <step> [<step> ...]
#   test:<pytest args>            python -m pytest <args> (commas -> spaces), -x -v, 120 s per test
#   bench:<name>:<bench args>     python bench.py <args> > <name>.json
#   smoke                         __graft_entry__.smoke()
#   trace:<name>:<bench args>     rocprofv3 --kernel-trace --stats over bench.py <args>
#   pmc:<name>:<ctrs>:<bench args> rocprofv3 --pmc <ctrs> (commas -> spaces) over bench.py <args>
#   py:<name>:<script args>       python -u <script args> > <name>.log
#   env:<VAR>=<value>             export VAR for the steps after it (env:<VAR>= unsets it)
# e.g. tools/run.sh r4a 'test:tests/test_gpu_counter.py' 'bench:c2c:--workload,c2c,--steps,5'
set -o pipefail
tag=$1
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
sp() { echo "${1//,/ }"; }
for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}
  echo "[run.sh] $(date +%T) $step" | tee -a "$out/steps.log"
  case $kind in
    test)
      # (commas separate arguments; '@' stands for a space inside one, e.g. -k,fuzz@or@wide)
      IFS=',' read -ra A <<< "$rest"
      for i in "${!A[@]}"; do A[$i]=${A[$i]//@/ }; done
      timeout -k 10 1000 python -u -m pytest "${A[@]}" -x -v --timeout 300 --timeout-method thread \
        > "$out/pytest_$(echo "$rest" | tr -c 'A-Za-z0-9_' _ | cut -c1-40).log" 2>&1 || { echo "[run.sh] FAILED $step"; exit 1; } ;;
    bench)
      name=${rest%%:*}; args=$(sp "${rest#*:}")
      timeout -k 10 600 python -u bench.py $args > "$out/$name.json" 2> "$out/$name.err" || { echo "[run.sh] FAILED $step"; tail -5 "$out/$name.err"; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { echo "[run.sh] FAILED smoke"; exit 1; } ;;
    trace)
      name=${rest%%:*}; args=$(sp "${rest#*:}")
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${name}_trace" -o run -- \
        python -u bench.py $args > "$out/${name}_trace.log" 2>&1 || { echo "[run.sh] FAILED $step"; exit 1; } ;;
    pmc)
      name=${rest%%:*}; r2=${rest#*:}; ctrs=$(sp "${r2%%:*}"); args=$(sp "${r2#*:}")
      timeout -s KILL 200 rocprofv3 --pmc $ctrs --output-format csv -d "$out/${name}_pmc" -o run -- \
        python -u bench.py $args > "$out/${name}_pmc.log" 2>&1 || { echo "[run.sh] FAILED $step"; exit 1; } ;;
    py)
      name=${rest%%:*}; args=$(sp "${rest#*:}")
      timeout -k 10 900 python -u $args > "$out/$name.log" 2>&1 || { echo "[run.sh] FAILED $step"; tail -5 "$out/$name.log"; exit 1; } ;;
    env)
      var=${rest%%=*}; val=${rest#*=}
      if [ -n "$val" ]; then export "$var=$val"; else unset "$var"; fi ;;
    *) echo "[run.sh] unknown step $step"; exit 2 ;;
  esac
done
echo "[run.sh] done" | tee -a "$out/steps.log"
