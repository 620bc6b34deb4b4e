"""Pin the counter workload's exact search at size with the CPU oracle (test infrastructure).

The reference checks a counter run as ONE whole-history `:linear` search
(/root/reference/src/jepsen/jgroups/workload/counter.clj:133-137, model :100-127). These
fixtures pin that search at sizes the GPU tests and bench use:

  c2c   C2's shape as a counter: 1 key x 5k ops, 16 clients, no crashes (~5 s)
  c2c4  the same history shape with 4 crashed ops anywhere in it (~75 s)
  c5x   C5's low-crash exact-search variant: 1M ops, 16 clients, 4 crashed ops in the first
        1 % ("exact search: <= ~15 crashed total"; hours on one thread)

Each config is checked once by the oracle on the build container's CPU (one thread, as Knossos
searches one history) and written to tests/golden/counter_<name>_oracle.json with the generator
call, the wall time and the host as provenance. tests/test_gpu.py compares the GPU search
against these files; tests/test_oracle.py checks that the generator still yields the history
each file was made from (entry count and a digest of the columns).

    python tests/golden/pin_counter.py c2c c2c4 c5x
"""
import hashlib
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

# name -> (generator call as text, the call)
GEN = {
    "c2c": ("synth.gen_config('c2c')", lambda: synth.gen_config("c2c")),
    "c2c4": ("synth.gen_counter(5000, 16, 0.0, 12345, n_crashed=4)",
             lambda: synth.gen_counter(5000, 16, 0.0, 12345, n_crashed=4)),
    "c5x": ("synth.gen_config('c5x')", lambda: synth.gen_config("c5x")),
}


def digest(h) -> str:
    """sha256 over the history's columns (the generator-drift check)."""
    m = hashlib.sha256()
    for col in (h.process, h.type, h.f, h.v0, h.v1, h.vflags):
        m.update(col.tobytes())
    return m.hexdigest()[:32]


def path_of(name: str) -> str:
    return os.path.join(HERE, f"counter_{name}_oracle.json")


def pin(name: str):
    import shutil
    import tempfile
    # a private copy of the oracle library, so rebuilding oracle/ meanwhile is harmless
    oracle.build()
    priv = os.path.join(tempfile.mkdtemp(prefix=f"pin_{name}_"), "liblincheck_oracle.so")
    shutil.copy(oracle.LIB, priv)
    oracle.LIB = priv
    call, gen = GEN[name]
    h = gen()
    t0 = time.time()
    r = oracle.check_one("counter", h)
    wall = time.time() - t0
    out = {
        "config": name,
        "generator": "lincheck." + call,
        "n_entries": int(h.n),
        "n_ops": int(h.n_ops()),
        "digest": digest(h),
        "valid": r["valid"],
        "err_code": r["err_code"],
        "fail_idx": r["fail_idx"],
        "prev_ok_idx": r["prev_ok_idx"],
        "explored": r["explored"],
        "max_frontier": r["max_frontier"],
        "n_returns": r["n_returns"],
        "final_frontier": r["final_frontier"],
        "provenance": {
            "command": f"python tests/golden/pin_counter.py {name}",
            "checker": "oracle/lincheck_oracle.c (oracle_check, one thread)",
            "wall_s": round(wall, 1),
            "host": platform.processor() or platform.machine(),
            "date": time.strftime("%Y-%m-%d"),
        },
    }
    with open(path_of(name), "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or ["c2c", "c2c4"]:
        pin(n)
