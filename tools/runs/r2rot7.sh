set -o pipefail
o=gpurun_out/r2rot7; mkdir -p $o
for r in 1 2; do
for cfg in "0.7 -1" "0.7 0" "0.45 0" "0.55 -1"; do
set -- $cfg
LC_PLAN_K=$1 LC_TEAM_ROT=$2 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e${r}_k$1_r$2.json 2> /dev/null || exit 1
done
done
for r in 1 2; do
for cfg in "0.7 -1" "0.45 -1" "0.7 0"; do
set -- $cfg
LC_PLAN_K=$1 LC_TEAM_ROT=$2 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/4 > $o/g${r}_k$1_r$2.json 2> /dev/null || exit 1
done
done
echo done
