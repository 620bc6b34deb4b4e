set -o pipefail
# r3ak: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the big kernel on C2 and C4, then their bench lines
o=gpurun_out/r3ak; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in c2 c4; do
P="python -u bench.py --workload $w --no-cpu --e2e-reps 0 --steps 1 --warmup 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/${w}_pmc_fetch -o run -- $P > $o/${w}_pmc.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/${w}_pmc_write -o run -- $P >> $o/${w}_pmc.log 2>&1 || exit 1
done
echo done
