set -o pipefail
o=gpurun_out/r2y; mkdir -p $o
for w in c3 c1 c2; do
timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/$w.json 2> $o/$w.err || exit 1
done
timeout -k 10 200 python -u bench.py --workload c4 --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c4.json 2> $o/c4.err || exit 1
for r in 0 1 2 3 4 5 6 7; do
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e$r.json 2> $o/e$r.err || exit 1
done
for r in 0 1; do
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/2 > $o/f$r.json 2> $o/f$r.err || exit 1
done
echo done
