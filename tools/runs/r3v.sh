set -o pipefail
# r3v: C3's batch plan with MID histories up to width 12 / 13 / 14 (LC_MID_MAXW), 2 passes
o=gpurun_out/r3v; mkdir -p $o
for rep in 1 2; do
for mw in 14 13 12; do
LC_MID_MAXW=$mw timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 >> $o/c3_mid$mw.json 2> /dev/null || exit 1
done
done
LC_MID_MAXW=13 LC_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_mid13_debug.json 2> $o/c3_mid13_debug.log || exit 1
echo done
