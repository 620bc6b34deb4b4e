export LC_DEBUG=1
timeout -k 10 300 python -u - > gpurun_out/r5e/dbg.log 2>&1 <<'PY'
import sys, os
sys.path[:0] = ["jepsen-jgroups-raft_amd", "tools"]
from lincheck import _lib, synth
import c3_team_alone as C
h = synth.gen_config("c3")
for i in range(2):
    _lib.check(1, 0, h)
    print("batch kernel_ms", _lib.check_stats(0)["kernel_ms"], file=sys.stderr, flush=True)
w = [C.live_width(h, k) for k in range(h.n_hist)]
wide = [k for k in range(h.n_hist) if w[k] >= 17]
for i in range(2):
    _lib.check(1, 0, h.select(wide))
    print("teams kernel_ms", _lib.check_stats(0)["kernel_ms"], file=sys.stderr, flush=True)
_lib.check(1, 0, h.select([258]))
print("alone258 kernel_ms", _lib.check_stats(0)["kernel_ms"], file=sys.stderr, flush=True)
PY
