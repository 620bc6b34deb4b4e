set -o pipefail
# r3an: C2 on 12-slot tiles without tagged mirrors (tokens) / without double-buffered tiles / without pipelined WAVE/MID
o=gpurun_out/r3an; mkdir -p $o
run() { tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_$tag.json 2> $o/c2_$tag.log || exit 1; }
run def
run notag LC_PIPE=$((217039 & ~256))
run nodbl LC_PIPE=$((217039 & ~512))
run def2
echo done
