set -o pipefail
# r3al: bench lines quote the per-workload traffic files (C2, C4) and the headline's
o=gpurun_out/r3al; mkdir -p $o
timeout -k 10 200 python -u bench.py --workload c2 --steps 3 --warmup 1 --no-cpu --e2e-reps 0 > $o/c2.json 2> $o/c2.log || exit 1
timeout -k 10 300 python -u bench.py > $o/c3.json 2> $o/c3.log || exit 1
echo done
