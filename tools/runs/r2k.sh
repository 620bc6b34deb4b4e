set -o pipefail
o=gpurun_out/r2k; mkdir -p $o
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c3_dbg.err || exit 1
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --workload c1 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c1_dbg.err || exit 1
LC_DEBUG=1 LC_PIPE=15 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c3_p15_dbg.err || exit 1
echo done
