"""why do C3's tile teams run slower per step inside the batch than alone?

Runs (warm, best of 3 lc_check calls each, one process on the GPU box):
  batch      all 1000 C3 keys (the bench's workload)
  alone:k    each of the widest keys by itself (a tile team with the chip to itself)
  teams      only the keys that take tile teams, together (no BLOCK / WAVE pools beside them)
and prints one JSON line per run with the kernel time and the slowest history's steps, width and
microseconds per step (lc_check_stats 39..41).

    python tools/c3_team_alone.py [--top 4]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jepsen-jgroups-raft_amd"), os.path.join(ROOT, "tests")]
from lincheck import _lib, synth, history as H  # noqa: E402


def live_width(h, k):
    """encode.cpp's live width (lowest-free-first slots, crashed ops keep theirs; :fail never enters)."""
    a, b = int(h.off[k]), int(h.off[k + 1])
    comp, pend = {}, {}
    for i in range(a, b):
        p = int(h.process[i])
        if h.type[i] == 0:
            pend[p] = i
        else:
            comp[pend.pop(p)] = int(h.type[i])
    live, width, slots = 0, 0, {}
    for i in range(a, b):
        p = int(h.process[i])
        if h.type[i] == 0:
            if comp.get(i) == 2:
                continue
            slots[p] = i
            live += 1
            width = max(width, live)
        elif int(h.type[i]) != 3 and p in slots and slots[p] is not None:
            # :ok returns free the slot; :info keeps it for ever
            live -= 1
            slots[p] = None
    return width


def run(name, h, reps=3):
    best, st = None, None
    for _ in range(reps + 1):
        _lib.check(1, 0, h)
        s = _lib.check_stats(0)
        if best is None or s["kernel_ms"] < best:
            best, st = s["kernel_ms"], s
    us, steps = st["slowest_history_us"], st["slowest_history_steps"]
    print(json.dumps({"run": name, "n_hist": int(h.n_hist), "kernel_ms": round(best, 3),
                      "slowest_us": round(us, 1), "slowest_steps": int(steps),
                      "slowest_width": int(st["slowest_history_width"]),
                      "us_per_step": round(us / max(1, steps), 2),
                      "dense_histories": int(st["dense_histories"])}), flush=True)
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=4)
    a = ap.parse_args()
    t0 = time.time()
    h = synth.gen_config("c3")
    widths = [live_width(h, k) for k in range(h.n_hist)]
    order = sorted(range(h.n_hist), key=lambda k: -widths[k])
    print(json.dumps({"widths_top": [(k, widths[k]) for k in order[:16]], "gen_s": round(time.time() - t0, 1)}), flush=True)
    run("batch", h)
    for k in order[:a.top]:
        run(f"alone:{k}:w{widths[k]}", h.select([k]))
    wide = [k for k in range(h.n_hist) if widths[k] >= 17]
    run(f"teams:{len(wide)}", h.select(wide))
    run("batch", h)


if __name__ == "__main__":
    main()
