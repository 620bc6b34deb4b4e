set -o pipefail
o=gpurun_out/r2ks; mkdir -p $o
for k in 0.5 0.7 0.9 1.2; do
for sh in 2/4 1/4 3/8 2/8 1/8 0/2 1/2; do
n=$(echo $sh | tr / _)
LC_PLAN_K=$k timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_k$k.json 2> /dev/null || exit 1
done
done
echo done
