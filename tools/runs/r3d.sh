set -o pipefail
# r3d: full GPU suite (invocation arrays skipped for dense-built histories, REG fixpoint for
# steps <= 7 slots), C3 end to end, A/B of LC_PIPE 1999 vs 4047 on C1 and C3 (alternating)
o=gpurun_out/r3d; mkdir -p $o
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
LC_PHASES=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e2e-reps 9 > $o/c3.json 2> $o/c3.err || exit 1
for i in 1 2 3; do
for pp in 1999 4047; do
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --workload c1 --steps 50 --warmup 10 --no-cpu --e2e-reps 9 > $o/c1_${pp}_$i.json 2> /dev/null || exit 1
LC_PIPE=$pp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e-reps 0 > $o/c3_${pp}_$i.json 2> /dev/null || exit 1
done
done
echo done
