set -o pipefail
o=gpurun_out/r2l3; mkdir -p $o
for r in 2 1; do
LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate $r/8 > /dev/null 2> $o/e${r}_dbg.err || exit 1
done
echo done
