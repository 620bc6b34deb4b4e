set -o pipefail
# r3w: C3 batch plan: LC_MID_MAXW {13, 14} x the team-estimate multiplier LC_PLAN_TM {1.0, 1.15, 1.3}, 2 passes
o=gpurun_out/r3w; mkdir -p $o
for rep in 1 2; do
for mw in 13 14; do
for tm in 1.0 1.15 1.3; do
LC_MID_MAXW=$mw LC_PLAN_TM=$tm timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_mid${mw}_tm$tm.json 2> /dev/null || exit 1
done
done
done
echo done
