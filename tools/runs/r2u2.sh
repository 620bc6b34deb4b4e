set -o pipefail
o=gpurun_out/r2u2; mkdir -p $o
LC_PART_FLOW=2 timeout -k 10 100 python -u bench.py --workload c2 --partition --steps 1 --warmup 0 --no-cpu --e2e-reps 0 > $o/c2p.json 2> $o/c2p.err
echo rc=$?
