import json, os, sys
sys.path[:0] = ["jepsen-jgroups-raft_amd", "tests/golden"]
from lincheck import _lib
import pin_wide
for n in ("ramp11s", "ramp10c17", "ramp11c17"):
    model, _, gen = pin_wide.GEN[n]
    h = gen()
    for rep in range(2):
        g = _lib.check(1, 0, h)
        st = _lib.check_stats()
    print(json.dumps({"name": n, "digest": pin_wide.digest(h), "valid": int(g["valid"][0]), "fail_idx": int(g["fail_idx"][0]),
                      "explored": int(g["explored"][0]), "wide": int(st["wide_histories"]), "dense": int(st["dense_histories"]),
                      "kernel_ms": st["kernel_ms"]}), flush=True)
