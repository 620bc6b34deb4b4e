set -o pipefail
o=gpurun_out/r2c3; mkdir -p $o
for pp in 975 909 911; do
LC_PIPE=$pp timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu --e2e-reps 0 > $o/c1_$pp.json 2> /dev/null || exit 1
done
echo done
