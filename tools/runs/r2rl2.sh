set -o pipefail
o=gpurun_out/r2rl2; mkdir -p $o
for t in 14 15 16; do
for sh in 2/4 1/4 2/8 3/8 0/2; do
n=$(echo $sh | tr / _)
LC_TEAM_ROT_LB=$t timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $sh > $o/s${n}_t$t.json 2> /dev/null || exit 1
done
done
echo done
