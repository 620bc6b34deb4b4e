#!/usr/bin/env python3
"""One process, no children: check the crash ramp's history K (default 16, width 30) with
lc_check twice (the second call warm) and print the HBM-table kernel's figures. For profiling
the HBM-table kernel under rocprofv3 (tools/crash_ramp.py starts child processes, which must not
run under the profiler)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jepsen-jgroups-raft_amd"))
from lincheck import _lib, synth  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 16
h = synth.gen_register(2000, 16, 0.002, 0x5EED4000 + k, n_crashed=k)
for rep in range(2):
    g = _lib.check(1, 0, h)
    st = _lib.check_stats()
print(json.dumps({"crashed": k, "valid": int(g["valid"][0]), "explored": int(g["explored"][0]),
                  "wide_histories": st["wide_histories"], "wide_ms": st["wide_ms"],
                  "wide_alg_gb": st["wide_hbm_bytes"] / 1e9,
                  "wide_alg_gbps": st["wide_hbm_bytes"] / st["wide_ms"] / 1e6 if st["wide_ms"] else None}))
