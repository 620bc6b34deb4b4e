set -o pipefail
o=gpurun_out/r2k2; mkdir -p $o
for c in 22 23 25; do
timeout -k 10 150 python -u bench.py --workload c4 --partition --capacity-log2 $c --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > $o/c4p_$c.json 2> $o/c4p_$c.err || exit 1
done
echo done
