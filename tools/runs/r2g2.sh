set -o pipefail
o=gpurun_out/r2g2; mkdir -p $o
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 2/4 > $o/g2.json 2> $o/g2.err || exit 1
LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 3/8 > $o/e3.json 2> $o/e3.err || exit 1
echo done
