set -o pipefail
o=gpurun_out/r2o; mkdir -p $o
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_dbg.json 2> $o/c3_dbg.err || exit 1
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --workload c2 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_dbg.json 2> $o/c2_dbg.err || exit 1
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 3/8 > $o/e3_dbg.json 2> $o/e3_dbg.err || exit 1
echo done
