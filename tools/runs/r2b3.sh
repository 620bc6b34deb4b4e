set -o pipefail
o=gpurun_out/r2b3; mkdir -p $o
for pp in 975 911; do
LC_PIPE=$pp timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu --e2e-reps 0 > $o/c1_$pp.json 2> /dev/null || exit 1
done
LC_DEBUG=1 timeout -k 10 100 python -u bench.py --workload c1 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c1_dbg.err || exit 1
echo done
