set -o pipefail
o=gpurun_out/r2o3; mkdir -p $o
for v in seq par; do
L=""; [ $v = par ] && L="$PWD/abtest/liblincheck_par.so"
LC_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_$v.json 2> /dev/null || exit 1
LC_LIB=$L timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --e2e-reps 0 > $o/c2_$v.json 2> /dev/null || exit 1
LC_LIB=$L timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/8 > $o/e2_$v.json 2> /dev/null || exit 1
LC_LIB=$L timeout -k 10 100 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu --e2e-reps 0 > $o/c1_$v.json 2> /dev/null || exit 1
done
echo done
