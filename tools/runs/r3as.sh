set -o pipefail
# r3as: 8-way C3 shares with chain plans also rotating their 12/13-slot teams (LC_TEAM_ROT_CHAIN_MIN=12) vs default
o=gpurun_out/r3as; mkdir -p $o
for v in def m12; do
if [ $v = m12 ]; then export LC_TEAM_ROT_CHAIN_MIN=12; else unset LC_TEAM_ROT_CHAIN_MIN; fi
for r in 0 1 2 3 4 5 6 7; do
timeout -k 10 200 python -u bench.py --emulate $r/8 --steps 5 --warmup 1 --no-cpu --e2e-reps 0 >> $o/c3e_$v.json 2>> $o/c3e_$v.log || exit 1
done
done
echo done
