set -o pipefail
# r3ab: why were C1's histories slower one per workgroup? LC_DEBUG stamps in both modes
o=gpurun_out/r3ab; mkdir -p $o
for pp in 217039 479183; do
LC_PIPE=$pp LC_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c1 --steps 3 --warmup 1 --no-cpu --e2e-reps 0 > $o/c1_$pp.json 2> $o/c1_$pp.log || exit 1
done
echo done
