set -o pipefail
o=gpurun_out/r2t3; mkdir -p $o
for x in 1.57 1.2 0.9; do
LC_PLAN_X=$x timeout -k 10 120 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_x$x.json 2> /dev/null || exit 1
LC_PLAN_X=$x timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_x$x.json 2> /dev/null || exit 1
for s in 0/2 1/2 1/4 2/4 1/8 2/8 3/8; do
n=$(echo $s | tr / _)
LC_PLAN_X=$x timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $s > $o/e${n}_x$x.json 2> /dev/null || exit 1
done
done
echo done
