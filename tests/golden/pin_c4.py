"""Pin C4's full-size verdict and explored count with the CPU oracle (test infrastructure).

C4 (BASELINE configs[3]): one 100k-op cas-register history, 16 clients, crashed :info ops
(synth.gen_config("c4")). The GPU paths (dense tile team, grid kernel, partitioned search) all
report the same explored count; this script settles it with the oracle on the build container's
CPU, once (~25 min on one thread), and writes tests/golden/c4_oracle.json with the command,
the wall time and the host as provenance. tests/test_gpu.py compares every C4 path against
that fixture.

    python tests/golden/pin_c4.py
"""
import json
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "jepsen-jgroups-raft_amd"))

import oracle  # noqa: E402
from lincheck import synth  # noqa: E402


def main():
    # run from a private copy of the oracle library, so rebuilding oracle/ meanwhile is harmless
    import shutil
    import tempfile
    oracle.build()
    priv = os.path.join(tempfile.mkdtemp(prefix="pin_c4_"), "liblincheck_oracle.so")
    shutil.copy(oracle.LIB, priv)
    oracle.LIB = priv
    h = synth.gen_config("c4")
    t0 = time.time()
    r = oracle.check_one("cas-register", h)
    wall = time.time() - t0
    out = {
        "config": "c4",
        "generator": "lincheck.synth.gen_config('c4')",
        "n_entries": int(h.n),
        "n_ops": int(h.n_ops()),
        "valid": r["valid"],
        "err_code": r["err_code"],
        "fail_idx": r["fail_idx"],
        "prev_ok_idx": r["prev_ok_idx"],
        "explored": r["explored"],
        "max_frontier": r["max_frontier"],
        "n_returns": r["n_returns"],
        "final_frontier": r["final_frontier"],
        "provenance": {
            "command": "python tests/golden/pin_c4.py",
            "checker": "oracle/lincheck_oracle.c (oracle_check, one thread)",
            "wall_s": round(wall, 1),
            "host": platform.processor() or platform.machine(),
            "date": time.strftime("%Y-%m-%d"),
        },
    }
    with open(os.path.join(HERE, "c4_oracle.json"), "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
