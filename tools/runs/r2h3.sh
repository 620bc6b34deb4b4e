set -o pipefail
o=gpurun_out/r2h3; mkdir -p $o
for v in b4 b2; do
L=""; [ $v = b2 ] && L="$PWD/abtest/liblincheck_b2.so"
LC_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_$v.json 2> /dev/null || exit 1
LC_LIB=$L timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_$v.json 2> /dev/null || exit 1
LC_LIB=$L timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/8 > $o/e2_$v.json 2> /dev/null || exit 1
LC_LIB=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4_$v.json 2> /dev/null || exit 1
done
echo done
