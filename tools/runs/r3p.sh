set -o pipefail
# r3p: LC_PLAN_ROT=1 around the batch factor 0.6 (is 10.9 ms a stable optimum?), with its team plan;
# C2 unrotated at tile sizes 13..16
o=${O:-gpurun_out/r3p}; mkdir -p $o
for rep in 1 2; do
for kb in 0.5 0.55 0.6 0.65 0.7; do
LC_PLAN_ROT=1 LC_PLAN_KB=$kb timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_r1_k$kb.json 2> /dev/null || exit 1
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_default.json 2> /dev/null || exit 1
done
for kb in 0.55 0.6 0.65; do
LC_PLAN_ROT=1 LC_PLAN_KB=$kb LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_r1_k${kb}_debug.json 2> $o/c3_r1_k${kb}_debug.log || exit 1
done
for lb in 14 15 16; do
LC_TILE_LBITS=$lb LC_TEAM_ROT=0 timeout -k 10 120 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_lb$lb.json 2> /dev/null || exit 1
done
echo done
