"""VERDICT r4 item 4, second probe: C3's widest key (258, width 21) alone with its tile size forced
(LC_TILE_LBITS = 14..17: 128..16 tiles) against the same key in the batch plan (lb 16, 32 tiles):
does the batch step cost come from the team's tile count or from the other teams beside it?
One JSON line per run (warm, best of 3)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jepsen-jgroups-raft_amd"), os.path.join(ROOT, "tools")]
from lincheck import _lib, synth  # noqa: E402
import c3_team_alone as C  # noqa: E402

h = synth.gen_config("c3")
w = [C.live_width(h, k) for k in range(h.n_hist)]
one = h.select([258])
wide = h.select([k for k in range(h.n_hist) if w[k] >= 17])
# argv: the runs (alone258, teams) and the tile sizes, e.g. alone258 plan,14,13,12
runs = sys.argv[1].split("+") if len(sys.argv) > 1 else ["alone258", "teams"]
lbs = [x if x != "plan" else "" for x in sys.argv[2].split("+")] if len(sys.argv) > 2 else ["", "17", "16", "15", "14"]
for name, hh in (("alone258", one), ("teams", wide)):
    if name not in runs:
        continue
    for lb in lbs:
        if lb:
            os.environ["LC_TILE_LBITS"] = lb
        elif "LC_TILE_LBITS" in os.environ:
            del os.environ["LC_TILE_LBITS"]
        C.run(f"{name}:lb{lb or 'plan'}", hh)
