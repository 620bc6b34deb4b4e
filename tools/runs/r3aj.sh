set -o pipefail
# r3aj: C2 on 12-slot tiles (the new default plan): rotations, global layers, XCD roles, credit window
o=gpurun_out/r3aj; mkdir -p $o
run() { tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2_$tag.json 2> $o/c2_$tag.log || exit 1; }
run def
run rot1 LC_TEAM_ROT=1
run rot2 LC_TEAM_ROT=2
run rot3 LC_TEAM_ROT=3
run rot9 LC_TEAM_ROT=9
run glob LC_PIPE=$((217039 | 8192))
run noxcd LC_PIPE=$((217039 & ~16384))
run cw8 LC_PIPE=$((217039 & ~131072))
run nocpre LC_PIPE=$((217039 & ~65536))
run lb11 LC_PLAN_LBMIN=11 LC_PLAN_X=0.9
echo done
