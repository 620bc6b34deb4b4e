set -o pipefail
o=gpurun_out/r2rl; mkdir -p $o
for i in 1 2; do
for t in 14 15 16; do
LC_TEAM_ROT_LB=$t timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_t${t}_$i.json 2> /dev/null || exit 1
done
done
echo done
