set -o pipefail
o=gpurun_out/r2c; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "dense or c3 or shards" > $o/pytest.log 2>&1 || exit 1
for cfg in "11 17" "15 17" "15 16" "15 15" "11 16"; do
  set -- $cfg
  LC_PIPE=$1 LC_TILE_LBITS=$2 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 > $o/c3_p$1_l$2.json 2> $o/c3_p$1_l$2.err || exit 1
  LC_PIPE=$1 LC_TILE_LBITS=$2 LC_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 1 --no-cpu --e2e-reps 0 > /dev/null 2> $o/c3_dbg_p$1_l$2.err || exit 1
  LC_PIPE=$1 LC_TILE_LBITS=$2 timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu --e2e-reps 0 --emulate 2/8 > $o/e2_p$1_l$2.json 2> /dev/null || exit 1
done
echo done
