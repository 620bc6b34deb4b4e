"""ctypes binding of liblincheck.so — the same C-ABI a JVM caller binds through JNA
(include/lincheck.h; INTEGRATION.md shows the JNA interface). There is deliberately no
CPU fallback: if the library or a HIP device is missing, calls raise."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LC_LIB") or os.path.join(HERE, "liblincheck.so")  # (LC_LIB: an A/B build)

# every symbol include/lincheck.h declares (tests check the exports)
EXPORTS = ("lc_abi_version", "lc_device_count", "lc_check", "lc_release", "lc_check_stats", "lc_shard_histories",
           "lc_shard_histories_by_cost",
           "lc_failure_configs",
           "lc_counter_bounds", "lc_plan_create", "lc_plan_run", "lc_plan_results",
           "lc_plan_stats", "lc_plan_destroy", "lc_bounds_plan_create", "lc_bounds_plan_sums",
           "lc_bounds_plan_run", "lc_bounds_plan_destroy", "lc_part_create", "lc_part_info",
           "lc_part_step_begin", "lc_part_expand", "lc_part_pack", "lc_part_absorb",
           "lc_part_step_end", "lc_part_results", "lc_part_run", "lc_part_destroy", "lc_part_check")
ABI_VERSION = 6
STATS_N = 44
STATS_NAMES = ("kernel_ms", "launches", "steps", "phases", "frontier_in", "candidates",
               "frontier_out", "closure_new", "config_bytes", "alg_bytes", "workgroups",
               "spill_inserts", "dense_histories", "dense_ms", "dense_big_ms", "dense_wave_ms",
               "dense_big_hbm_bytes", "dense_big_lds_bytes", "dense_wave_hbm_bytes",
               "dense_wave_lds_bytes", "create_encode_ms", "create_device_init_ms",
               "create_streams_ms", "create_upload_ms", "create_dense_streams_ms",
               "dense_big_frontier_in", "dense_big_frontier_out", "dense_big_explored",
               "dense_wave_frontier_in", "dense_wave_frontier_out", "dense_wave_explored",
               "wide_histories", "wide_ms", "wide_hbm_bytes",
               "ctab_histories", "ctab_ms", "ctab_frontier_in", "ctab_frontier_out", "ctab_explored",
               "slowest_history_us", "slowest_history_steps", "slowest_history_width",
               "ctab_team_histories", "wide_slabs")

P = C.c_void_p
I8P = C.POINTER(C.c_int8)
_lib = None


class LincheckError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LincheckError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; "
                            "g.build()'` (the checker has no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    L.lc_abi_version.restype = C.c_int32
    L.lc_device_count.restype = C.c_int32
    L.lc_check.argtypes = [C.c_int32, C.c_int64, C.c_int32] + [P] * 8 + \
        [C.c_int32, C.c_int64, C.c_int32] + [P] * 6 + [C.c_char_p, C.c_int32]
    L.lc_check.restype = C.c_int32
    L.lc_release.argtypes = [C.c_int32]
    L.lc_release.restype = C.c_int32
    L.lc_check_stats.argtypes = [C.c_int32, P, C.c_int32]
    L.lc_check_stats.restype = C.c_int32
    L.lc_shard_histories.argtypes = [C.c_int32, P, C.c_int32, P]
    L.lc_shard_histories_by_cost.argtypes = [C.c_int32, C.c_int64, C.c_int32] + [P] * 8 + \
        [C.c_int32, P, P, C.c_char_p, C.c_int32]
    L.lc_shard_histories_by_cost.restype = C.c_int32
    L.lc_shard_histories.restype = C.c_int32
    L.lc_failure_configs.argtypes = [C.c_int32, C.c_int32] + [P] * 9 + [C.c_char_p, C.c_int32]
    L.lc_failure_configs.restype = C.c_int32
    L.lc_counter_bounds.argtypes = [C.c_int64, C.c_int32] + [P] * 10 + [C.c_char_p, C.c_int32]
    L.lc_counter_bounds.restype = C.c_int32
    L.lc_plan_create.argtypes = [C.c_int32, C.c_int32, C.c_int64, C.c_int32] + [P] * 8 + \
        [C.c_int64, C.POINTER(C.c_void_p), C.c_char_p, C.c_int32]
    L.lc_plan_create.restype = C.c_int32
    L.lc_plan_run.argtypes = [P, C.c_char_p, C.c_int32]
    L.lc_plan_run.restype = C.c_int32
    L.lc_plan_results.argtypes = [P] * 7
    L.lc_plan_results.restype = C.c_int32
    L.lc_plan_stats.argtypes = [P, P, C.c_int32]
    L.lc_plan_stats.restype = C.c_int32
    L.lc_plan_destroy.argtypes = [P]
    L.lc_plan_destroy.restype = None
    L.lc_bounds_plan_create.argtypes = [C.c_int32, C.c_int64, C.c_int64] + [P] * 7 + \
        [C.c_int64, C.c_int64, C.POINTER(C.c_void_p), C.c_char_p, C.c_int32]
    L.lc_bounds_plan_create.restype = C.c_int32
    L.lc_bounds_plan_sums.argtypes = [P, P, C.c_char_p, C.c_int32]
    L.lc_bounds_plan_sums.restype = C.c_int32
    L.lc_bounds_plan_run.argtypes = [P] * 5 + [C.c_char_p, C.c_int32]
    L.lc_bounds_plan_run.restype = C.c_int32
    L.lc_bounds_plan_destroy.argtypes = [P]
    L.lc_bounds_plan_destroy.restype = None
    L.lc_part_create.argtypes = [C.c_int32, C.c_int32, C.c_int64, C.c_int64] + [P] * 7 + \
        [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p), C.c_char_p, C.c_int32]
    L.lc_part_create.restype = C.c_int32
    L.lc_part_info.argtypes = [P, P, C.c_int32]
    L.lc_part_info.restype = C.c_int32
    L.lc_part_step_begin.argtypes = [P, C.c_int64, P, C.c_char_p, C.c_int32]
    L.lc_part_step_begin.restype = C.c_int32
    L.lc_part_expand.argtypes = [P, P, P, C.c_char_p, C.c_int32]
    L.lc_part_expand.restype = C.c_int32
    L.lc_part_pack.argtypes = [P, P, P, C.c_int64, C.c_char_p, C.c_int32]
    L.lc_part_pack.restype = C.c_int32
    L.lc_part_absorb.argtypes = [P, P, P, C.c_int64, C.c_char_p, C.c_int32]
    L.lc_part_absorb.restype = C.c_int32
    L.lc_part_step_end.argtypes = [P, P, P, C.c_char_p, C.c_int32]
    L.lc_part_step_end.restype = C.c_int32
    L.lc_part_results.argtypes = [P, C.c_int64, P, P, C.c_char_p, C.c_int32]
    L.lc_part_results.restype = C.c_int32
    L.lc_part_run.argtypes = [P, P, C.c_int64, P, C.c_char_p, C.c_int32]
    L.lc_part_run.restype = C.c_int32
    L.lc_part_check.argtypes = [C.c_int32, C.c_int64, C.c_int64] + [P] * 7 + [C.c_int32, C.c_int32] + \
        [P] * 6 + [C.c_char_p, C.c_int32]
    L.lc_part_check.restype = C.c_int32
    L.lc_part_destroy.argtypes = [P]
    L.lc_part_destroy.restype = None
    if L.lc_abi_version() != ABI_VERSION:
        raise LincheckError("ABI version mismatch")
    _lib = L
    return L


def _p(a):
    # (the address as an int: half the cost of data_as, whose c_void_p object C1's 14 arrays paid
    # ~60 us per lc_check for; the arrays outlive the call)
    return None if a is None else a.ctypes.data


def _errbuf():
    return C.create_string_buffer(512)


def _raise(rc, buf, what):
    if rc != 0:
        raise LincheckError(f"{what} failed ({rc}): {buf.value.decode(errors='replace')}")


MODEL_KIND = {"cas-register": 1, "counter": 2}


def check(model_kind: int, init_value: int, h, n_gpus: int = 1, max_configs: int = 0,
          flags: int = 0):
    """Run lc_check on a lincheck.history.History. Returns a dict of numpy arrays."""
    L = load()
    n = h.n_hist
    out = {"valid": np.zeros(n, np.int8), "fail_idx": np.zeros(n, np.int64),
           "fail_inv": np.zeros(n, np.int64), "prev_ok": np.zeros(n, np.int64),
           "explored": np.zeros(n, np.int64), "err": np.zeros(n, np.int32)}
    buf = _errbuf()
    rc = L.lc_check(model_kind, init_value, n, _p(h.off), _p(h.index), _p(h.process), _p(h.type),
                    _p(h.f), _p(h.v0), _p(h.v1), _p(h.vflags), n_gpus, max_configs, flags,
                    _p(out["valid"]), _p(out["fail_idx"]), _p(out["fail_inv"]), _p(out["prev_ok"]),
                    _p(out["explored"]), _p(out["err"]), buf, len(buf))
    _raise(rc, buf, "lc_check")
    return out


def release(device: int = -1):
    """lc_release: free lc_check's cached per-device plan(s) and their device memory."""
    load().lc_release(device)


def check_stats(device: int = 0):
    """lc_check_stats: statistics of the last lc_check run on `device` (Plan.stats() names)."""
    s = np.zeros(STATS_N, np.float64)
    rc = load().lc_check_stats(device, _p(s), STATS_N)
    if rc != 0:
        raise LincheckError(f"lc_check_stats failed ({rc})")
    return dict(zip(STATS_NAMES, s.tolist()))


def shard_histories(h, n_shards: int) -> np.ndarray:
    """lc_shard_histories: the LPT split lc_check uses over n_shards (host only)."""
    out = np.zeros(max(h.n_hist, 1), np.int32)
    rc = load().lc_shard_histories(h.n_hist, _p(h.off), n_shards, _p(out))
    if rc != 0:
        raise LincheckError(f"lc_shard_histories failed ({rc})")
    return out[:h.n_hist]


def shard_histories_by_cost(model_kind: int, init_value: int, h, n_shards: int):
    """lc_shard_histories_by_cost: the split lc_check(n_gpus) uses -> (shard per history,
    modeled chain time per history in us). Host only."""
    out = np.zeros(max(h.n_hist, 1), np.int32)
    cost = np.zeros(max(h.n_hist, 1), np.float64)
    buf = _errbuf()
    rc = load().lc_shard_histories_by_cost(model_kind, init_value, h.n_hist, _p(h.off), _p(h.index),
                                           _p(h.process), _p(h.type), _p(h.f), _p(h.v0), _p(h.v1),
                                           _p(h.vflags), n_shards, _p(out), _p(cost), buf, len(buf))
    _raise(rc, buf, "lc_shard_histories_by_cost")
    return out[:h.n_hist], cost[:h.n_hist]


def failure_configs(hist: int, k: int = 10, with_last=False):
    """Pre-failure frontier of history `hist` of the last check() on this thread ->
    (configs [(value, linearized invocation :index tuple)], pending invocation :index list);
    with_last: + (per-config :last-op completion :index list, the frontier's newest)."""
    L = load()
    st = np.zeros(k, np.int64)
    nil = np.zeros(k, np.int8)
    lin = np.zeros(k * 64, np.int64)
    nlin = np.zeros(k, np.int32)
    last = np.zeros(k, np.int64)
    nout = np.zeros(1, np.int32)
    pend = np.zeros(64, np.int64)
    npend = np.zeros(1, np.int32)
    newest = np.zeros(1, np.int64)
    buf = _errbuf()
    rc = L.lc_failure_configs(hist, k, _p(st), _p(nil), _p(lin), _p(nlin), _p(last), _p(nout),
                              _p(pend), _p(npend), _p(newest), buf, len(buf))
    _raise(rc, buf, "lc_failure_configs")
    cfgs = []
    for i in range(int(nout[0])):
        cfgs.append((None if nil[i] else int(st[i]),
                     tuple(sorted(int(x) for x in lin[i * 64:i * 64 + nlin[i]]))))
    pending = [int(x) for x in pend[:npend[0]]]
    if with_last:
        return cfgs, pending, [int(x) for x in last[:nout[0]]], int(newest[0])
    return cfgs, pending


def part_check(h, hist: int = 0, n_ranks: int = 0, capacity_log2: int = 0):
    """lc_part_check: history `hist` of h with its frontier partitioned over n_ranks in-process
    ranks (peer copies between devices). Returns lc_check-shaped scalars."""
    L = load()
    b, e = int(h.off[hist]), int(h.off[hist + 1])
    keep = [np.ascontiguousarray(a[b:e]) for a in
            (h.index, h.process, h.type, h.f, h.v0, h.v1, h.vflags)]
    out = {"valid": np.zeros(1, np.int8), "fail_idx": np.zeros(1, np.int64),
           "fail_inv": np.zeros(1, np.int64), "prev_ok": np.zeros(1, np.int64),
           "explored": np.zeros(1, np.int64), "err": np.zeros(1, np.int32)}
    buf = _errbuf()
    rc = L.lc_part_check(1, 0, e - b, *[_p(a) for a in keep], n_ranks, capacity_log2,
                         _p(out["valid"]), _p(out["fail_idx"]), _p(out["fail_inv"]), _p(out["prev_ok"]),
                         _p(out["explored"]), _p(out["err"]), buf, len(buf))
    _raise(rc, buf, "lc_part_check")
    return out


def counter_bounds(init_value: int, h):
    L = load()
    ok = np.zeros(h.n_hist, np.int8)
    bad = np.zeros(h.n_hist, np.int64)
    buf = _errbuf()
    rc = L.lc_counter_bounds(init_value, h.n_hist, _p(h.off), _p(h.index), _p(h.process),
                             _p(h.type), _p(h.f), _p(h.v0), _p(h.v1), _p(h.vflags), _p(ok),
                             _p(bad), buf, len(buf))
    _raise(rc, buf, "lc_counter_bounds")
    return ok, bad


class Plan:
    """Device-resident encoded histories (lc_plan_*): run() times only the search."""

    def __init__(self, model_kind: int, init_value: int, h, device: int = 0, max_configs: int = 0):
        L = load()
        self._L = L
        self.n_hist = h.n_hist
        handle = C.c_void_p()
        buf = _errbuf()
        rc = L.lc_plan_create(device, model_kind, init_value, h.n_hist, _p(h.off), _p(h.index),
                              _p(h.process), _p(h.type), _p(h.f), _p(h.v0), _p(h.v1),
                              _p(h.vflags), max_configs, C.byref(handle), buf, len(buf))
        _raise(rc, buf, "lc_plan_create")
        self._h = handle

    def run(self):
        buf = _errbuf()
        _raise(self._L.lc_plan_run(self._h, buf, len(buf)), buf, "lc_plan_run")

    def results(self):
        n = self.n_hist
        out = {"valid": np.zeros(n, np.int8), "fail_idx": np.zeros(n, np.int64),
               "fail_inv": np.zeros(n, np.int64), "prev_ok": np.zeros(n, np.int64),
               "explored": np.zeros(n, np.int64), "err": np.zeros(n, np.int32)}
        self._L.lc_plan_results(self._h, _p(out["valid"]), _p(out["fail_idx"]), _p(out["fail_inv"]),
                                _p(out["prev_ok"]), _p(out["explored"]), _p(out["err"]))
        return out

    def stats(self):
        s = np.zeros(STATS_N, np.float64)
        self._L.lc_plan_stats(self._h, _p(s), STATS_N)
        return dict(zip(STATS_NAMES, s.tolist()))

    def close(self):
        if self._h:
            self._L.lc_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BoundsPlan:
    """Device-resident counter bounds scan over one history, or over the shard of it whose
    observations complete in entries [own_begin, own_end) (lc_bounds_plan_*). Sharded use:
    sums() on every shard, exchange (lincheck.shard.exclusive_sums), then run(excl)."""

    def __init__(self, init_value: int, h, hist: int = 0, own=None, device: int = 0):
        L = load()
        self._L = L
        b, e = int(h.off[hist]), int(h.off[hist + 1])
        n = e - b
        own_begin, own_end = own if own is not None else (0, n)
        self.own = (own_begin, own_end)
        sl = slice(b, e)
        self._keep = [np.ascontiguousarray(a[sl]) for a in
                      (h.index, h.process, h.type, h.f, h.v0, h.v1, h.vflags)]
        handle = C.c_void_p()
        buf = _errbuf()
        rc = L.lc_bounds_plan_create(device, init_value, n, *[_p(a) for a in self._keep], own_begin,
                                     own_end, C.byref(handle), buf, len(buf))
        _raise(rc, buf, "lc_bounds_plan_create")
        self._h = handle
        self._keep = None

    def sums(self):
        out = np.zeros(5, np.int64)
        buf = _errbuf()
        _raise(self._L.lc_bounds_plan_sums(self._h, _p(out), buf, len(buf)), buf, "lc_bounds_plan_sums")
        return out

    def run(self, excl=None):
        """-> (ok, bad :index or -1, kernel ms)"""
        ok = np.zeros(1, np.int8)
        bad = np.zeros(1, np.int64)
        ms = np.zeros(1, np.float64)
        ex = None if excl is None else np.ascontiguousarray(excl, dtype=np.int64)
        buf = _errbuf()
        rc = self._L.lc_bounds_plan_run(self._h, _p(ex), _p(ok), _p(bad), _p(ms), buf, len(buf))
        _raise(rc, buf, "lc_bounds_plan_run")
        return bool(ok[0]), int(bad[0]), float(ms[0])

    def close(self):
        if self._h:
            self._L.lc_bounds_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PartPlan:
    """One rank's part of a single cas-register history whose frontier is partitioned over
    `world` ranks by config hash (lc_part_*, SURVEY §8(e) axis 2). Driven level by level by
    lincheck.partition.search, which runs the collectives. Buffers are torch tensors on the
    plan's device (or None where the C-ABI allows NULL); `stream` is a hipStream_t handle."""

    H_CAPACITY = -7

    def __init__(self, h, hist: int = 0, rank: int = 0, world: int = 1, device: int = 0,
                 capacity_log2: int = 0):
        L = load()
        self._L = L
        self.rank, self.world = rank, world
        b, e = int(h.off[hist]), int(h.off[hist + 1])
        keep = [np.ascontiguousarray(a[b:e]) for a in
                (h.index, h.process, h.type, h.f, h.v0, h.v1, h.vflags)]
        handle = C.c_void_p()
        buf = _errbuf()
        rc = L.lc_part_create(device, 1, 0, e - b, *[_p(a) for a in keep], rank, world,
                              capacity_log2, C.byref(handle), buf, len(buf))
        _raise(rc, buf, "lc_part_create")
        self._h = handle
        info = np.zeros(6, np.int64)
        L.lc_part_info(self._h, _p(info), 6)
        self.n_steps, self.err, self.mask_bits, self.state_bits, self.n_ops, self.list_cap = \
            (int(x) for x in info)
        self._counts = np.zeros(world, np.int64)

    def stats(self):
        """kernel time (ms, HIP events on the caller's stream) and algorithmic HBM bytes so far"""
        info = np.zeros(8, np.int64)
        self._L.lc_part_info(self._h, _p(info), 8)
        return {"kernel_ms": float(info[6]) / 1e6, "alg_bytes": float(info[7])}

    def _call(self, fn, *args):
        buf = _errbuf()
        rc = fn(self._h, *args, buf, len(buf))
        if rc == self.H_CAPACITY:
            raise CapacityError(buf.value.decode(errors="replace"))
        _raise(rc, buf, fn.__name__)

    def step_begin(self, t: int, stream=None):
        self._call(self._L.lc_part_step_begin, t, stream)

    def expand(self, stream=None):
        self._call(self._L.lc_part_expand, stream, _p(self._counts))
        return self._counts.copy()

    def pack(self, dst, stream=None):
        self._call(self._L.lc_part_pack, stream, dst.data_ptr(), dst.numel())

    def absorb(self, recv, n: int, stream=None):
        self._call(self._L.lc_part_absorb, stream, None if recv is None else recv.data_ptr(), n)

    def step_end(self, stream=None) -> int:
        out = np.zeros(1, np.int64)
        self._call(self._L.lc_part_step_end, stream, _p(out))
        return int(out[0])

    def run(self, stream=None, max_steps: int = -1):
        """World 1, device-resident level loop (lc_part_run) on a fresh plan ->
        (steps run, first failing step or -1, BFS levels, explored)."""
        out = np.zeros(4, np.int64)
        self._call(self._L.lc_part_run, stream, max_steps, _p(out))
        return tuple(int(x) for x in out)

    def results(self, t: int, stream=None):
        """-> (this rank's explored, fail :index, its invocation's :index, previous :ok's)"""
        out = np.zeros(4, np.int64)
        self._call(self._L.lc_part_results, t, stream, _p(out))
        return tuple(int(x) for x in out)

    def close(self):
        if self._h:
            self._L.lc_part_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CapacityError(LincheckError):
    """The frontier outgrew the plan's capacity (LC_H_CAPACITY: verdict :unknown)."""
