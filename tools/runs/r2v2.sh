set -o pipefail
o=gpurun_out/r2v2; mkdir -p $o
for w in c3 c2 c1; do
timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/$w.json 2> /dev/null || exit 1
done
timeout -k 10 200 python -u bench.py --workload c4 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4.json 2> /dev/null || exit 1
for sh in 0/2 1/2 0/4 1/4 2/4 3/4 0/8 1/8 2/8 3/8 4/8 5/8 6/8 7/8; do
n=$(echo $sh | tr / _)
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}.json 2> /dev/null || exit 1
done
echo done
