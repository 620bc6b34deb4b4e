#!/usr/bin/env python3
"""The crash ramp of SURVEY §8(d), config C4: "calibrate p_info so the CPU oracle finishes, then
ramp up and report where each side breaks".

A crashed (:info) write or cas stays pending for ever (knossos.history keeps it; the JIT search
may linearize it at any later point or never), so every crashed op adds a slot that is live for
the rest of the history and can double the frontier. This script generates one cas-register
history per crash count K (`synth.gen_register(n_crashed=K)`: exactly K write/cas ops time out,
drawn from the first 20 % of the ops, so they are pending for most of the history) and checks it

  * on the CPU: the C oracle (one thread, test infrastructure: the CPU side of the comparison),
    in a child process with a wall-clock limit;
  * on the GPU: `lc_check` (the product path: dense closure tables while the live width is
    <= 24, the grid kernel beyond), each K in a child process with a wall-clock limit;
  * optionally `lc_part_check` at one rank (--part: the partitioned hash-set search).

The CPU legs all run before anything touches the GPU (the children are spawned, not forked).
Output: one JSON line per K (stdout), with the explored counts compared where both sides finish.

  python tools/crash_ramp.py --ops 2000 --crashed 0,2,4,6,8,10,12 --cpu-timeout 120
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jepsen-jgroups-raft_amd"))
sys.path.insert(0, ROOT)

SEED0 = 0x5EED4000  # SURVEY §8(d) seeds: config 4


MODEL = "cas-register"  # --model counter: the counter workload's ramp


def make(ops: int, clients: int, k: int, model: str = "cas-register"):
    """K crashed ops in the first 20 %: write/cas for a register; for a counter the timed-out
    add / *-and-get ops of counter.clj:118-119,126-127 (client.clj:52-63 reports them :info)."""
    from lincheck import synth
    if model == "counter":
        return synth.gen_counter(ops, clients, 0.0, SEED0 + 0x100 + k, n_crashed=k, crash_span=0.2)
    return synth.gen_register(ops, clients, 0.002, SEED0 + k, n_crashed=k)


def width_of(h) -> int:
    """Most ops pending at once as the search sees them: an op that completes :fail never enters
    it, a crashed (:info) one stays pending for ever (the encoder's live width, `encode.cpp`)."""
    import numpy as np
    t = np.asarray(h.type)
    p = np.asarray(h.process)
    fails, open_ = set(), {}
    for i in range(len(t)):  # which invocations end :fail
        if t[i] == 0:
            open_[int(p[i])] = i
        elif int(p[i]) in open_:
            if t[i] == 2:
                fails.add(open_[int(p[i])])
            del open_[int(p[i])]
    live, best, pend = 0, 0, {}
    for i in range(len(t)):
        if t[i] == 0:
            if i in fails:
                continue
            pend[int(p[i])] = True
            live += 1
            best = max(best, live)
        elif t[i] == 1 and pend.pop(int(p[i]), None):
            live -= 1
    return best


def cpu_leg(ops, clients, k, model, q):
    from oracle import oracle
    h = make(ops, clients, k, model)
    t = time.perf_counter()
    r = oracle.check_one(model, h)
    q.put({"wall_s": time.perf_counter() - t, "valid": int(r["valid"]), "explored": int(r["explored"]),
           "max_frontier": int(r.get("max_frontier", -1))})


def gpu_leg(ops, clients, k, part, part_cap, model, q):
    from lincheck import _lib
    h = make(ops, clients, k, model)
    kind = _lib.MODEL_KIND[model]
    out = {}
    t = time.perf_counter()
    r = _lib.check(kind, 0, h)
    out["lc_check"] = {"wall_s": time.perf_counter() - t, "valid": int(r["valid"][0]),
                       "explored": int(r["explored"][0]), "err": int(r["err"][0])}
    st = _lib.check_stats()
    out["lc_check"]["path"] = ("wide (HBM tables)" if st.get("wide_histories", 0) > 0
                               else "counter tile team" if st.get("ctab_team_histories", 0) > 0
                               else "counter tables" if st.get("ctab_histories", 0) > 0
                               else "dense" if st.get("dense_histories", 0) > 0 else "grid")
    out["lc_check"]["kernel_ms"] = st.get("kernel_ms")
    if st.get("wide_histories", 0) > 0:  # HBM-table kernel: algorithmic bytes / its time vs 8 TB/s
        out["lc_check"]["wide_ms"] = st["wide_ms"]
        out["lc_check"]["wide_alg_gb"] = st["wide_hbm_bytes"] / 1e9
        out["lc_check"]["wide_alg_gbps"] = st["wide_hbm_bytes"] / st["wide_ms"] / 1e6 if st["wide_ms"] else None
    if out["lc_check"]["wall_s"] < 30:  # a second (warm) run: the device's first-use cost is gone
        t = time.perf_counter()
        _lib.check(kind, 0, h)
        out["lc_check"]["wall_warm_s"] = time.perf_counter() - t
    if part:
        t = time.perf_counter()
        try:
            p = _lib.part_check(h, 0, 1, part_cap)
            out["lc_part_check"] = {"wall_s": time.perf_counter() - t, "valid": int(p["valid"][0]),
                                    "explored": int(p["explored"][0]), "err": int(p["err"][0])}
        except Exception as e:  # capacity errors come back as :unknown; anything else is reported
            out["lc_part_check"] = {"error": str(e)[:200]}
    q.put(out)


def run_child(target, args, timeout):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=target, args=args + (q,))
    t = time.perf_counter()
    p.start()
    p.join(timeout)
    if p.is_alive():
        p.terminate()
        p.join(10)
        if p.is_alive():
            p.kill()
            p.join()
        return {"timeout_s": timeout, "wall_s": time.perf_counter() - t}
    try:
        return q.get(timeout=5)
    except Exception:
        return {"error": f"child exited with {p.exitcode}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", type=int, default=2000)
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--crashed", default="0,2,4,6,8,10,12")
    ap.add_argument("--cpu-timeout", type=float, default=120.0)
    ap.add_argument("--gpu-timeout", type=float, default=120.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--part", action="store_true")
    ap.add_argument("--part-cap", type=int, default=0, help="lc_part_check capacity_log2 (0: default)")
    ap.add_argument("--model", default="cas-register", choices=("cas-register", "counter"))
    a = ap.parse_args()
    ks = [int(x) for x in a.crashed.replace("+", ",").split(",") if x]  # ("+": tools/run.sh splits commas)
    rows = {}
    for k in ks:
        h = make(a.ops, a.clients, k, a.model)
        rows[k] = {"model": a.model, "crashed": k, "ops": a.ops, "clients": a.clients, "width": width_of(h),
                   "entries": int(h.n)}
    if not a.no_cpu:  # every CPU leg first: nothing in this process has touched the GPU yet
        for k in ks:  # (stops at the first K past the limit: where the CPU side breaks)
            rows[k]["cpu_oracle_1thread"] = run_child(cpu_leg, (a.ops, a.clients, k, a.model), a.cpu_timeout)
            print(f"[ramp] K={k} cpu {rows[k]['cpu_oracle_1thread']}", file=sys.stderr, flush=True)
            if "timeout_s" in rows[k]["cpu_oracle_1thread"]:
                break
    if not a.no_gpu:
        for k in ks:
            rows[k]["gpu"] = run_child(gpu_leg, (a.ops, a.clients, k, a.part, a.part_cap, a.model), a.gpu_timeout)
            print(f"[ramp] K={k} gpu {rows[k]['gpu']}", file=sys.stderr, flush=True)
            if "timeout_s" in rows[k]["gpu"] or "error" in rows[k]["gpu"]:
                break
    for k in ks:
        r = rows[k]
        c, g = r.get("cpu_oracle_1thread", {}), r.get("gpu", {}).get("lc_check", {})
        if "explored" in c and "explored" in g:
            r["explored_equal"] = c["explored"] == g["explored"] and c["valid"] == g["valid"]
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
