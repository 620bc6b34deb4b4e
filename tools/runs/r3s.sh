set -o pipefail
# r3s: the batch plan's team-estimate multiplier LC_PLAN_TM on C3 (2 alternating passes), with
# the team plan and pool ends at 1.0 and 1.5
o=gpurun_out/r3s; mkdir -p $o
for rep in 1 2; do
for tm in 1.0 1.2 1.4 1.6 1.8; do
LC_PLAN_TM=$tm timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_tm$tm.json 2> /dev/null || exit 1
done
done
for tm in 1.0 1.5; do
LC_PLAN_TM=$tm LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_tm${tm}_debug.json 2> $o/c3_tm${tm}_debug.log || exit 1
done
echo done
