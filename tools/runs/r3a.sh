set -o pipefail
# r3a: GPU suite (new failure-report tags, env-knob reset, lc_release), smoke, default bench,
# then ONE rocprofv3 pass of the partitioned C2 run with the maps dump (exit-crash diagnosis)
o=gpurun_out/r3a; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu > $o/c3.json 2> $o/c3.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
LC_MAPS_DUMP=$PWD/$o/part_maps.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/part_trace -o run -- python -u bench.py --workload c2 --partition --scale 0.3 --steps 1 --warmup 0 > $o/part_trace.log 2>&1
echo "part trace rc=$?" >> $o/part_trace.log
echo done
