"""Counter tile teams on the GPU box: the team size T (LC_CTAB_TEAM_T; 0 = one workgroup) swept
on c2c (width 16), c2c4 (width 20, 5k steps) and c5x (width 20, 1M steps), warm lc_check kernel
times and explored counts (the same for every T). One JSON line per case.

    python tools/ctab_team_sweep.py c2c=0+1+2+3 c2c4=0+1+2+3+4 c5x=2+3+4
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jepsen-jgroups-raft_amd")]
from lincheck import _lib, synth  # noqa: E402

GEN = {"c2c": lambda: synth.gen_config("c2c"),
       "c2c4": lambda: synth.gen_counter(5000, 16, 0.0, 12345, n_crashed=4),
       "c5x": lambda: synth.gen_config("c5x")}


def main(args):
    for a in args:
        name, ts = a.split("=")
        h = GEN[name]()
        for T in [int(x) for x in ts.split("+")]:
            os.environ["LC_CTAB_TEAM"] = "1" if T > 0 else "0"
            os.environ["LC_CTAB_TEAM_MINW"] = "1"
            os.environ["LC_CTAB_TEAM_T"] = str(T)
            reps = 1 if name == "c5x" else 3
            best, g, st = None, None, None
            for _ in range(reps + (0 if name == "c5x" else 1)):
                t0 = time.perf_counter()
                g = _lib.check(2, 0, h)
                wall = time.perf_counter() - t0
                st = _lib.check_stats(0)
                k = st["ctab_ms"]
                best = k if best is None else min(best, k)
            print(json.dumps({"config": name, "T": T, "kernel_ms": best, "wall_s": wall,
                              "valid": int(g["valid"][0]), "explored": int(g["explored"][0])}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
