set -o pipefail
o=gpurun_out/r2mid; mkdir -p $o
for sh in 2/4 3/4 1/4 0/4 2/8 3/8 1/8 6/8 0/2 1/2; do
n=$(echo $sh | tr / _)
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_def.json 2> /dev/null || exit 1
LC_MID_MAXW=12 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_m12.json 2> /dev/null || exit 1
LC_PIPE=335 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_nomid.json 2> /dev/null || exit 1
done
echo done
