set -o pipefail
o=gpurun_out/r2i; mkdir -p $o
for c in 17 19 21 23 25; do
timeout -k 10 200 python -u bench.py --workload c2 --partition --capacity-log2 $c --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2p_$c.json 2> $o/c2p_$c.err || exit 1
done
echo done
