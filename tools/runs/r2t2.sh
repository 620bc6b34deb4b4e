set -o pipefail
o=gpurun_out/r2t2; mkdir -p $o
LC_PART_FLOW=2 timeout -k 10 240 python -u -m pytest tests/test_gpu.py -x -v --timeout 100 --timeout-method thread -k "partitioned_world1_vs_oracle and flow or c2_slice or capacity_is_unknown and flow or stage_retry and flow" > $o/pytest.log 2>&1 || exit 1
LC_PART_FLOW=2 timeout -k 10 100 python -u bench.py --workload c2 --partition --steps 2 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2p.json 2> $o/c2p.err || exit 1
LC_PART_FLOW=2 timeout -k 10 150 python -u bench.py --workload c4 --partition --capacity-log2 25 --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > $o/c4p.json 2> $o/c4p.err || exit 1
echo done
