set -o pipefail
o=gpurun_out/r2b; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "dense or kats or c1 or c3 or random or c2_full or shards" > $o/pytest.log 2>&1 || exit 1
for pipe in 11 43; do
  LC_PIPE=$pipe timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 1 > $o/c3_p$pipe.json 2> $o/c3_p$pipe.err || exit 1
  LC_PIPE=$pipe LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c3_dbg_p$pipe.err || exit 1
  LC_PIPE=$pipe timeout -k 10 120 python -u bench.py --workload c1 --steps 20 --warmup 5 --no-cpu --e2e-reps 1 > $o/c1_p$pipe.json 2> $o/c1_p$pipe.err || exit 1
  LC_PIPE=$pipe timeout -k 10 120 python -u bench.py --workload c2 --steps 5 --warmup 2 --no-cpu --e2e-reps 1 > $o/c2_p$pipe.json 2> $o/c2_p$pipe.err || exit 1
done
echo done
