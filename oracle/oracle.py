"""ctypes wrapper of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module;
the product (jepsen-jgroups-raft_amd/lincheck + liblincheck.so) never does. See
lincheck_oracle.c for the restated reference functions and the parity-pinning status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liblincheck_oracle.so")


class OracleResult(C.Structure):
    _fields_ = [("valid", C.c_int32), ("err_code", C.c_int32), ("fail_idx", C.c_int64),
                ("fail_inv_idx", C.c_int64), ("prev_ok_idx", C.c_int64),
                ("explored", C.c_int64), ("max_frontier", C.c_int64),
                ("n_returns", C.c_int64), ("final_frontier", C.c_int64),
                ("n_fail_cfgs", C.c_int64), ("n_pending_at_fail", C.c_int32),
                ("_pad", C.c_int32), ("wall_ns", C.c_int64), ("pending_inv_idx", C.c_int64 * 64),
                ("err", C.c_char * 128)]

    def as_dict(self):
        return {"valid": self.valid, "err_code": self.err_code, "fail_idx": self.fail_idx,
                "fail_inv_idx": self.fail_inv_idx, "prev_ok_idx": self.prev_ok_idx,
                "explored": self.explored, "max_frontier": self.max_frontier,
                "n_returns": self.n_returns, "final_frontier": self.final_frontier,
                "n_fail_cfgs": self.n_fail_cfgs, "wall_ns": self.wall_ns,
                "err": self.err.decode()}


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.c_void_p
        L.oracle_check.argtypes = [C.c_int32, C.c_int64, C.c_int64] + [P] * 7 + \
            [C.c_int64, C.POINTER(OracleResult), C.c_int64, P, P, P, P]
        L.oracle_check.restype = C.c_int32
        L.oracle_check_many.argtypes = [C.c_int32, C.c_int64, C.c_int32] + [P] * 8 + \
            [C.c_int64, C.c_int32, C.POINTER(OracleResult)]
        L.oracle_check_many.restype = C.c_int32
        L.oracle_counter_bounds.argtypes = [C.c_int64, C.c_int64] + [P] * 7 + [C.POINTER(C.c_int64)]
        L.oracle_counter_bounds.restype = C.c_int32
        L.oracle_result_size.restype = C.c_int32
        assert L.oracle_result_size() == C.sizeof(OracleResult)
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


MODEL = {"cas-register": 1, "register": 1, "counter": 2, "leader": 3}


def check_one(model: str, h, init_value: int = 0, max_configs: int = 0, with_configs=False):
    """Check history h (a lincheck.history.History with one sub-history)."""
    L = lib()
    r = OracleResult()
    n = h.n
    cap = 1 << 20 if with_configs else 0
    cv = np.zeros(max(cap, 1), np.int64)
    cn = np.zeros(max(cap, 1), np.int8)
    cm = np.zeros(max(cap, 1), np.uint64)
    cl = np.zeros(max(cap, 1), np.int64)
    L.oracle_check(MODEL[model], init_value, n, _p(h.index), _p(h.process), _p(h.type),
                   _p(h.f), _p(h.v0), _p(h.v1), _p(h.vflags), max_configs, C.byref(r),
                   cap, _p(cv), _p(cn), _p(cm), _p(cl))
    d = r.as_dict()
    if with_configs and r.valid == 0:
        k = min(r.n_fail_cfgs, cap)
        pend = [r.pending_inv_idx[b] for b in range(r.n_pending_at_fail)]
        cfgs = set()
        last = {}
        for a in range(k):
            lin = tuple(sorted(pend[b] for b in range(len(pend)) if (int(cm[a]) >> b) & 1))
            c = (None if cn[a] else int(cv[a]), lin)
            cfgs.add(c)
            last[c] = int(cl[a])
        d["fail_configs"] = cfgs
        d["fail_last_op"] = last  # config -> :index of its :last-op's :ok completion (-1: none)
        d["pending_inv_idx"] = pend
    return d


def check_many(model: str, h, init_value: int = 0, max_configs: int = 0, n_threads: int = 0):
    L = lib()
    if n_threads <= 0:  # the process's CPU share where the environment states it (16 on a GPU box)
        n_threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or os.cpu_count() or 1
    res = (OracleResult * max(h.n_hist, 1))()
    L.oracle_check_many(MODEL[model], init_value, h.n_hist, _p(h.off), _p(h.index),
                        _p(h.process), _p(h.type), _p(h.f), _p(h.v0), _p(h.v1), _p(h.vflags),
                        max_configs, n_threads, res)
    return [res[i].as_dict() for i in range(h.n_hist)]


def counter_bounds(h, init_value: int = 0):
    L = lib()
    bad = C.c_int64(-1)
    ok = L.oracle_counter_bounds(init_value, h.n, _p(h.index), _p(h.process), _p(h.type),
                                 _p(h.f), _p(h.v0), _p(h.v1), _p(h.vflags), C.byref(bad))
    return bool(ok), bad.value
