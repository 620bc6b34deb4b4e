set -o pipefail
# r3ar: C3 (batch plan) with the rotation threshold moved (LC_TEAM_ROT_LB, default 16), interleaved, twice
o=gpurun_out/r3ar; mkdir -p $o
for rep in 1 2; do
for v in 16 14 15 17; do
LC_TEAM_ROT_LB=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --e2e-reps 0 >> $o/c3_rot$v.json 2>> $o/c3.log || exit 1
done
done
echo done
