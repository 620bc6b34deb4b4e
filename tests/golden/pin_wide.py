"""Pin real wide frontiers and full-size INVALID runs with the CPU oracle (test infrastructure).

VERDICT r4 item 1. Every earlier full-size fixture was a valid history, and the HBM tables
(csrc/wide.hip, live widths 25..35) were pinned only on bases padded with never-applying calls.
These fixtures are the oracle's answers on:

  ramp13      the crash ramp's K = 13 history (tools/crash_ramp.py: 2,000 ops, 16 clients,
              13 crashed write/cas in the first 20 %): live width 27, ~7 G configs explored;
              runs on the HBM tables
  ramp14      K = 14 (width 27, ~17 G configs)
  ramp16      K = 16 (width 30, ~59 G configs; hours, and only if its frontier fits memory)
  ramp11s     r5: a 1,000-op ramp history, 16 clients, K = 11: live width 25 (HBM tables)
  ramp10c17   r5: 1,000 ops, 17 clients, K = 10: width 25
  ramp11c17   r5: 1,000 ops, 17 clients, K = 11: width 26
  ramp13x50   ramp13 with one :ok read perturbed at 50 % of the history: the pipelined HBM-table
              kernel must stop mid-history with later steps already in flight
  c4x15       C4 (100k ops, width 23: the rotated 128-tile team) with one read perturbed at 15 %
              (r5: the changed value stays explainable, so the history is still valid: a second
              full-size C4 count, 10,994,825,722 configs)
  c4x15n      r5: C4 with its first read after 15 % returning 7, a value never written: invalid,
              so the team stops mid-history
  c5xx2       c5x (the 1M-op counter, width 20: the counter closure tables) perturbed at 2 %

Each is checked once by the oracle on the build container's CPU (one thread, as Knossos searches
one history; the reference's invalid-verdict shape is raft_test.clj:29-65) and written to
tests/golden/wide_<name>_oracle.json with the generator call, a digest of the columns, the wall
time and the host. tests/test_gpu_pins.py compares the GPU search against them (verdict, the
failing :index triple and the explored count); tests/test_oracle.py checks that the generator
still yields the history each file was made from.

    python tests/golden/pin_wide.py ramp13 ramp13x50 ...
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

from lincheck import synth  # noqa: E402

RAMP_SEED0 = 0x5EED4000  # tools/crash_ramp.py SEED0 (SURVEY §8(d) seeds, config 4)


def read_never_written(h, at_frac: float):
    """h with its first :ok scalar read from entry at_frac * n returning 7, a value the register
    generator never writes (its domain is 0..4): invalid at that read, so the search stops there."""
    import numpy as np
    from lincheck import history as H
    t, f, vf = np.asarray(h.type), np.asarray(h.f), np.asarray(h.vflags)
    start = int(at_frac * h.n)
    j = start + int(np.nonzero((t[start:] == 1) & (f[start:] == 0) & (vf[start:] == H.V_SCALAR))[0][0])
    v0 = np.array(h.v0, copy=True)
    v0[j] = 7
    return H.from_columns(np.array(h.index, copy=True), np.array(h.process, copy=True), t.copy(), f.copy(), v0,
                          np.array(h.v1, copy=True), vf.copy())


def ramp(k: int):
    return synth.gen_register(2000, 16, 0.002, RAMP_SEED0 + k, n_crashed=k)


# name -> (model, generator call as text, the call)
GEN = {
    "ramp13": ("cas-register", "synth.gen_register(2000, 16, 0.002, 0x5EED4000 + 13, n_crashed=13)",
               lambda: ramp(13)),
    "ramp14": ("cas-register", "synth.gen_register(2000, 16, 0.002, 0x5EED4000 + 14, n_crashed=14)",
               lambda: ramp(14)),
    "ramp16": ("cas-register", "synth.gen_register(2000, 16, 0.002, 0x5EED4000 + 16, n_crashed=16)",
               lambda: ramp(16)),
    # r5: real wide frontiers the oracle can finish in the build container (the K = 13 history
    # needs > 36 GB: OOM-killed here): 1,000-op ramp histories just past the tile teams
    "ramp11s": ("cas-register", "synth.gen_register(1000, 16, 0.002, 0x5EED4000 + 11, n_crashed=11)",
                lambda: synth.gen_register(1000, 16, 0.002, RAMP_SEED0 + 11, n_crashed=11)),
    "ramp10c17": ("cas-register", "synth.gen_register(1000, 17, 0.002, 0x5EED4000 + 10, n_crashed=10)",
                  lambda: synth.gen_register(1000, 17, 0.002, RAMP_SEED0 + 10, n_crashed=10)),
    "ramp11c17": ("cas-register", "synth.gen_register(1000, 17, 0.002, 0x5EED4000 + 11, n_crashed=11)",
                  lambda: synth.gen_register(1000, 17, 0.002, RAMP_SEED0 + 11, n_crashed=11)),
    "ramp13x50": ("cas-register",
                  "synth.perturb_read(synth.gen_register(2000, 16, 0.002, 0x5EED4000 + 13, "
                  "n_crashed=13), 0.5, 'cas-register', 50)",
                  lambda: synth.perturb_read(ramp(13), 0.5, "cas-register", 50)),
    "c4x15": ("cas-register", "synth.perturb_read(synth.gen_config('c4'), 0.15, 'cas-register', 15)",
              lambda: synth.perturb_read(synth.gen_config("c4"), 0.15, "cas-register", 15)),
    "c4x15n": ("cas-register", "read_never_written(synth.gen_config('c4'), 0.15)",
               lambda: read_never_written(synth.gen_config("c4"), 0.15)),
    "c5xx2": ("counter", "synth.perturb_read(synth.gen_config('c5x'), 0.02, 'counter', 2)",
              lambda: synth.perturb_read(synth.gen_config("c5x"), 0.02, "counter", 2)),
}


def digest(h) -> str:
    """sha256 over the history's columns (the generator-drift check)."""
    m = hashlib.sha256()
    for col in (h.process, h.type, h.f, h.v0, h.v1, h.vflags):
        m.update(col.tobytes())
    return m.hexdigest()[:32]


def path_of(name: str) -> str:
    return os.path.join(HERE, f"wide_{name}_oracle.json")


def pin(name: str):
    import shutil
    import tempfile
    import oracle
    # a private copy of the oracle library, so rebuilding oracle/ meanwhile is harmless
    oracle.build()
    priv = os.path.join(tempfile.mkdtemp(prefix=f"pin_{name}_"), "liblincheck_oracle.so")
    shutil.copy(oracle.LIB, priv)
    oracle.LIB = priv
    model, call, gen = GEN[name]
    h = gen()
    t0 = time.time()
    r = oracle.check_one(model, h)
    wall = time.time() - t0
    out = {
        "config": name,
        "model": model,
        "generator": "lincheck." + call,
        "n_entries": int(h.n),
        "n_ops": int(h.n_ops()),
        "digest": digest(h),
        "valid": r["valid"],
        "err_code": r["err_code"],
        "fail_idx": r["fail_idx"],
        "fail_inv_idx": r["fail_inv_idx"],
        "prev_ok_idx": r["prev_ok_idx"],
        "explored": r["explored"],
        "max_frontier": r["max_frontier"],
        "n_returns": r["n_returns"],
        "final_frontier": r["final_frontier"],
        "provenance": {
            "command": f"python tests/golden/pin_wide.py {name}",
            "checker": "oracle/lincheck_oracle.c (oracle_check, one thread)",
            "wall_s": round(wall, 1),
            "host": platform.processor() or platform.machine(),
            "date": time.strftime("%Y-%m-%d"),
        },
    }
    if r["err_code"] != 0:
        print(json.dumps(out), flush=True)
        raise SystemExit(f"{name}: the oracle did not finish ({r['err_code']}): not written")
    with open(path_of(name), "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:]:
        pin(n)
