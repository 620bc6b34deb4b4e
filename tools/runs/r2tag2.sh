set -o pipefail
o=gpurun_out/r2tag2; mkdir -p $o
for i in 1 2 3; do
for pp in 207 463; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_${pp}_$i.json 2> /dev/null || exit 1
done
done
for pp in 207 463; do
for r in 1 2; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_$pp.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/4 > $o/g${r}_$pp.json 2> /dev/null || exit 1
done
done
echo done
