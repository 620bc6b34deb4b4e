set -o pipefail
o=gpurun_out/r2v; mkdir -p $o
for w in 12 13 14; do
LC_MID_MAXW=$w LC_PIPE=207 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_207_w$w.json 2> $o/c3_207_w$w.err || exit 1
done
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_79.json 2> $o/c3_79.err || exit 1
LC_MID_MAXW=13 LC_PIPE=207 LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_207_dbg.json 2> $o/c3_207_dbg.err || exit 1
echo done
