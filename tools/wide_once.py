#!/usr/bin/env python3
"""One process, no children: check the crash ramp's history K (default 16, width 30) with
lc_check twice (cold, then warm) and print the HBM-table kernel's figures. For profiling the
HBM-table kernels under rocprofv3 (tools/crash_ramp.py starts child processes, which must not
run under the profiler): the register ramp (wide_pipe_kernel; slabs from width 36) or, with
`counter`, the counter ramp (wctr_pipe_kernel).

    python tools/wide_once.py 21                # cas-register, K = 21 (width 36, two slabs)
    python tools/wide_once.py 20 counter        # counter, K = 20 (width 34)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jepsen-jgroups-raft_amd"), os.path.join(ROOT, "tools")]
from lincheck import _lib  # noqa: E402
import crash_ramp  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 16
model = sys.argv[2] if len(sys.argv) > 2 else "cas-register"
h = crash_ramp.make(2000, 16, k, model)
out = {"model": model, "crashed": k, "width": crash_ramp.width_of(h)}
for rep in ("cold", "warm"):
    g = _lib.check(_lib.MODEL_KIND[model], 0, h)
    st = _lib.check_stats()
    out[rep] = {"valid": int(g["valid"][0]), "explored": int(g["explored"][0]),
                "wide_histories": st["wide_histories"], "wide_ms": st["wide_ms"],
                "wide_alg_gb": st["wide_hbm_bytes"] / 1e9,
                "wide_alg_gbps": st["wide_hbm_bytes"] / st["wide_ms"] / 1e6 if st["wide_ms"] else None,
                "slabs": int(st["wide_slabs"])}
print(json.dumps(out), flush=True)
