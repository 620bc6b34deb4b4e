set -o pipefail
o=gpurun_out/r2p3; mkdir -p $o
for rep in 1 2; do
for pp in 1743 1999; do
LC_PIPE=$pp timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_${pp}_$rep.json 2> /dev/null || exit 1
done
done
echo done
