set -o pipefail
o=gpurun_out/r2cd; mkdir -p $o
for sh in 0/2 1/2 0/4 1/4 2/4 3/4 0/8 1/8 2/8 3/8 4/8 5/8 6/8 7/8; do
n=$(echo $sh | tr / _)
LC_MID_MAXW=12 LC_PLAN_K=1.0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_c.json 2> /dev/null || exit 1
LC_PIPE=335 LC_PLAN_K=1.0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_d.json 2> /dev/null || exit 1
LC_PLAN_K=1.0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_k.json 2> /dev/null || exit 1
done
echo done
