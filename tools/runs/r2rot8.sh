set -o pipefail
o=gpurun_out/r2rot8; mkdir -p $o
for cfg in "0.45 0" "0.45 -1" "0.35 0" "0.55 0"; do
set -- $cfg
LC_PLAN_K=$1 LC_TEAM_ROT=$2 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_k$1_r$2.json 2> /dev/null || exit 1
done
echo done
