"""Counter closure tables on the GPU box: parity spot checks against the oracle and warm
lc_check times on C2's shape as a counter (c2c), with crashed ops (c2c4) and on the grid kernel
(LC_CTAB_MAXW=0) for comparison. One JSON line per case.

    python tools/ctab_probe.py [c2c c2c4 grid c5x ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jepsen-jgroups-raft_amd"), os.path.join(ROOT, "oracle")]
for a in list(sys.argv[1:]):  # lib=<suffix>: an A/B build lincheck/liblincheck_<suffix>.so
    if a.startswith("lib="):
        os.environ["LC_LIB"] = os.path.join(ROOT, "jepsen-jgroups-raft_amd", "lincheck", f"liblincheck_{a[4:]}.so")
        sys.argv.remove(a)

import oracle  # noqa: E402  (checker of the spot checks)
from lincheck import _lib, history as H, synth  # noqa: E402


def timed(h, reps=3):
    ts = []
    g = None
    for _ in range(reps):
        t0 = time.perf_counter()
        g = _lib.check(2, 0, h)
        ts.append(time.perf_counter() - t0)
    st = _lib.check_stats(0)
    return g, min(ts), st


def fixture(name):
    p = os.path.join(ROOT, "tests", "golden", f"counter_{name}_oracle.json")
    return json.load(open(p)) if os.path.exists(p) else None


def main(cases):
    # small parity first (a wrong kernel shows here before the big cases)
    hs = [synth.gen_counter(60 + 7 * t, 1 + t % 12, 0.05, 100 + t, invalid=(t % 3 == 0)) for t in range(24)]
    h = H.concat(hs)
    g = _lib.check(2, 0, h)
    exp = oracle.check_many("counter", h, n_threads=8)
    bad = [k for k in range(h.n_hist) if int(g["valid"][k]) != exp[k]["valid"] or
           int(g["explored"][k]) != exp[k]["explored"] or int(g["fail_idx"][k]) != exp[k]["fail_idx"]]
    print(json.dumps({"case": "small", "n": h.n_hist, "mismatch": bad[:10],
                      "ctab": _lib.check_stats(0)["ctab_histories"]}), flush=True)
    if bad:
        k = bad[0]
        print(json.dumps({"first_bad": k, "gpu": [int(g[x][k]) for x in ("valid", "fail_idx", "explored")],
                          "oracle": [exp[k][x] for x in ("valid", "fail_idx", "explored")]}), flush=True)
        return 1
    for c in cases:
        if c in ("c2c", "c2c4", "c5x", "grid"):
            name = "c2c" if c == "grid" else c
            if name == "c2c4":
                h = synth.gen_counter(5000, 16, 0.0, 12345, n_crashed=4)
            else:
                h = synth.gen_config(name)
            if c == "grid":
                os.environ["LC_CTAB_MAXW"] = "0"
            g, t, st = timed(h, reps=3 if name != "c5x" else 2)
            os.environ.pop("LC_CTAB_MAXW", None)
            fx = fixture(name)
            print(json.dumps({"case": c, "lib": os.environ.get("LC_LIB", "default"), "ops": h.n_ops(), "valid": int(g["valid"][0]),
                              "explored": int(g["explored"][0]),
                              "fixture_explored": fx and fx["explored"],
                              "match": fx is not None and int(g["explored"][0]) == fx["explored"] and
                              int(g["valid"][0]) == fx["valid"],
                              "lc_check_ms": round(t * 1e3, 3), "kernel_ms": round(st["kernel_ms"], 3),
                              "ctab_ms": round(st["ctab_ms"], 3), "ctab": st["ctab_histories"],
                              "encode_ms": round(st["create_encode_ms"], 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or ["c2c", "c2c4", "grid"]))
