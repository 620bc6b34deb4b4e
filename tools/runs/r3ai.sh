set -o pipefail
# r3ai: default planner vs LC_PLAN_X=1.2 LC_PLAN_LBMIN=12 on the 8-way C3 shares (no LC_DEBUG), twice each
o=gpurun_out/r3ai; mkdir -p $o
for rep in 1 2; do
for v in def x12; do
if [ $v = x12 ]; then export LC_PLAN_X=1.2 LC_PLAN_LBMIN=12; else unset LC_PLAN_X LC_PLAN_LBMIN; fi
for r in 0 1 2 3 4 5 6 7; do
timeout -k 10 200 python -u bench.py --emulate $r/8 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 >> $o/c3e_$v.json 2>> $o/c3e_$v.log || exit 1
done
timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 >> $o/c2_$v.json 2>> $o/c2_$v.log || exit 1
done
done
echo done
