set -o pipefail
o=gpurun_out/r2bh; mkdir -p $o
for i in 1 2; do
for sh in 0/2 1/2; do
n=$(echo $sh | tr / _)
LC_BATCH_HIST=600 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_600_$i.json 2> /dev/null || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_400_$i.json 2> /dev/null || exit 1
done
done
echo done
