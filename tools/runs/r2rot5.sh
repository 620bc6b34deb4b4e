set -o pipefail
o=gpurun_out/r2rot5; mkdir -p $o
for k in 0.2 0.3 0.35 0.4 0.45; do
LC_PLAN_K=$k timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_k$k.json 2> $o/c3_k$k.err || exit 1
done
LC_PLAN_K=0.4 LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > $o/c3_dbg.json 2> $o/c3_dbg.err || exit 1
for r in 1 2 3; do
LC_PLAN_K=0.4 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e$r.json 2> $o/e$r.err || exit 1
done
for w in c2 c4 c1; do
LC_PLAN_K=0.4 timeout -k 10 200 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu --e2e-reps 0 > $o/$w.json 2> $o/$w.err || exit 1
done
echo done
