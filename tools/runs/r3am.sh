set -o pipefail
# r3am: C3's batch plan at the new team-bit cost: LC_PLAN_KB x LC_PLAN_TM, interleaved, twice
o=gpurun_out/r3am; mkdir -p $o
for rep in 1 2; do
for kb in 0.35 0.45 0.6; do
for tm in 1.0 1.3; do
LC_PLAN_KB=$kb LC_PLAN_TM=$tm timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --e2e-reps 0 >> $o/c3_kb${kb}_tm${tm}.json 2>> $o/c3.log || exit 1
done
done
done
echo done
