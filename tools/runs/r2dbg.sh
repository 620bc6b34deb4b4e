set -o pipefail
o=gpurun_out/r2dbg; mkdir -p $o
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c2 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2.json 2> $o/c2.err || exit 1
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > $o/c4.json 2> $o/c4.err || exit 1
echo done
