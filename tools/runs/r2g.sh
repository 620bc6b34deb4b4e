set -o pipefail
o=gpurun_out/r2g; mkdir -p $o
for k in 1 2 3 4; do
  for pipe in 15 31; do
    LC_PLAN_K=$k LC_PIPE=$pipe timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_k${k}_p$pipe.json 2> /dev/null || exit 1
  done
done
LC_PLAN_K=3 LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c3_k3_dbg.err || exit 1
for r in 0 1 2 3 4 5 6 7; do
  LC_PLAN_K=3 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/8 > $o/e$r.json 2> /dev/null || exit 1
done
for r in 0 1 2 3; do
  LC_PLAN_K=3 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/4 > $o/f$r.json 2> /dev/null || exit 1
done
for r in 0 1; do
  LC_PLAN_K=3 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate $r/2 > $o/g$r.json 2> /dev/null || exit 1
done
LC_DEBUG=1 LC_PLAN_K=3 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 --emulate 5/8 > /dev/null 2> $o/e5_dbg.err || exit 1
echo done
