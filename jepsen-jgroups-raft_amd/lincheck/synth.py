"""Synthetic Jepsen histories of a simulated linearizable SUT.

Each client loops: invoke at t, latency ~ U(1,10) ticks, linearization point ~
U(invoke, complete); effects are applied to a ground-truth register/counter in
linearization-point order, so every generated history is linearizable unless
`invalid=True` perturbs one read.

Value domains follow the reference generators:
  * register: f mix 1/3 read/write/cas (register.clj:116), values U{0..4} (:21-34);
    a cas whose expected value does not match is a definite :fail (:84); CAS on a nil
    register fails (ReplicatedMap.java:37-48).
  * counter: f uniform over read/add/decr/add-and-get/decr-and-get (counter.clj:138),
    deltas U{0..4} (:15-38); *-and-get ok -> [delta new] (:91-93).
Error model (client.clj:52-63): with probability p_info a non-read op times out ->
:info (applied with probability 1/2, possibly after its completion time) and the client
continues under a fresh process id (p + n_clients); a timed-out read is :fail.
Seeds: seed = 0x5EED0000 + config_id*1000 + key.
"""
from __future__ import annotations

import numpy as np

from .history import History, V_NIL, V_PAIR, V_SCALAR, concat, from_columns, leader_id

F_READ, F_WRITE, F_CAS, F_ADD, F_DECR, F_AAG, F_DAG, F_INSPECT = range(8)
T_INV, T_OK, T_FAIL, T_INFO = range(4)


def seed_for(config_id: int, key: int) -> int:
    return 0x5EED0000 + config_id * 1000 + key


def _schedule(rng, n_ops, n_clients, p_info, fs, crash_idx=None):
    """Per-op timing for n_ops ops spread over n_clients back-to-back clients."""
    per = np.full(n_clients, n_ops // n_clients)
    per[: n_ops % n_clients] += 1
    client = np.repeat(np.arange(n_clients), per)
    lat = rng.uniform(1.0, 10.0, n_ops)
    gap = rng.uniform(0.0, 1.0, n_ops)
    inv = np.empty(n_ops)
    start = 0
    for c in range(n_clients):
        k = per[c]
        if k == 0:
            continue
        seg_lat, seg_gap = lat[start:start + k], gap[start:start + k]
        prev = np.concatenate(([0.0], np.cumsum(seg_lat + seg_gap)[:-1]))
        inv[start:start + k] = rng.uniform(0, 1) + prev + seg_gap
        start += k
    cmp_ = inv + lat
    lin = inv + rng.uniform(0.0, 1.0, n_ops) * lat
    crashed = (fs != F_READ) & (rng.uniform(size=n_ops) < p_info)
    if crash_idx is not None:  # exactly these (non-read) ops crash (the crash ramp)
        crashed = np.zeros(n_ops, bool)
        crashed[np.asarray(crash_idx, np.int64)] = True
    read_fail = (fs == F_READ) & (rng.uniform(size=n_ops) < p_info)
    applied_if_crashed = rng.uniform(size=n_ops) < 0.5
    # a crashed op may take effect late (after its completion time)
    lin = np.where(crashed, inv + rng.uniform(0.0, 3.0, n_ops) * lat, lin)
    return client, inv, cmp_, lin, crashed, read_fail, applied_if_crashed


def _emit(n_clients, client, inv, cmp_, typ, fs, inv_v, cmp_v, crashed):
    """Interleave invoke/completion events by time; assign process ids (fresh after :info)."""
    n = len(inv)
    # process id per op: the client's id bumps by n_clients after each crashed op
    order_c = np.lexsort((inv, client))
    proc = np.empty(n, np.int64)
    bump = np.zeros(n_clients, np.int64)
    for i in order_c:
        c = client[i]
        proc[i] = c + n_clients * bump[c]
        if crashed[i]:
            bump[c] += 1
    times = np.concatenate((inv, cmp_))
    kind = np.concatenate((np.zeros(n, np.int8), np.ones(n, np.int8)))
    opid = np.concatenate((np.arange(n), np.arange(n)))
    order = np.lexsort((kind, times))
    m = 2 * n
    out_t = np.empty(m, np.int8)
    out_p = np.empty(m, np.int32)
    out_f = np.empty(m, np.int8)
    out_vf = np.empty(m, np.int8)
    out_v0 = np.empty(m, np.int64)
    out_v1 = np.empty(m, np.int64)
    k_o, o_o = kind[order], opid[order]
    out_p[:] = proc[o_o]
    out_f[:] = fs[o_o]
    is_inv = k_o == 0
    out_t[:] = np.where(is_inv, T_INV, typ[o_o])
    vf_inv, a_inv, b_inv = inv_v
    vf_c, a_c, b_c = cmp_v
    out_vf[:] = np.where(is_inv, vf_inv[o_o], vf_c[o_o])
    out_v0[:] = np.where(is_inv, a_inv[o_o], a_c[o_o])
    out_v1[:] = np.where(is_inv, b_inv[o_o], b_c[o_o])
    return from_columns(np.arange(m), out_p, out_t, out_f, out_v0, out_v1, out_vf)


def gen_register(n_ops: int, n_clients: int, p_info: float, seed: int,
                 invalid: bool = False, n_crashed: int | None = None,
                 crash_span: float = 0.2) -> History:
    """n_crashed: exactly that many write/cas ops time out (:info), drawn uniformly from the
    first `crash_span` of the ops (the crash ramp); p_info then only makes reads
    :fail. Default (None): every non-read op crashes with probability p_info."""
    rng = np.random.default_rng(seed)
    fs = rng.integers(0, 3, n_ops).astype(np.int8)  # read / write / cas
    val = rng.integers(0, 5, n_ops)
    old = rng.integers(0, 5, n_ops)
    crash_idx = None
    if n_crashed is not None:
        span = np.nonzero(fs[:max(1, int(n_ops * crash_span))] != F_READ)[0]
        crash_idx = np.random.default_rng(seed ^ 0xC4A5).choice(span, min(n_crashed, len(span)), replace=False)
    client, inv, cmp_, lin, crashed, read_fail, app_c = _schedule(rng, n_ops, n_clients, p_info, fs,
                                                                  crash_idx)
    typ = np.full(n_ops, T_OK, np.int8)
    res = np.zeros(n_ops, np.int64)
    res_nil = np.zeros(n_ops, bool)
    state, nil = 0, True
    for i in np.argsort(lin, kind="stable"):
        f = fs[i]
        if f == F_READ:
            if read_fail[i]:
                typ[i] = T_FAIL
            else:
                res[i], res_nil[i] = state, nil
        elif f == F_WRITE:
            if crashed[i]:
                typ[i] = T_INFO
                if not app_c[i]:
                    continue
            state, nil = int(val[i]), False
        else:  # cas
            ok = (not nil) and state == old[i]
            if crashed[i]:
                typ[i] = T_INFO
                if ok and app_c[i]:
                    state = int(val[i])
            elif ok:
                state = int(val[i])
            else:
                typ[i] = T_FAIL
    if invalid:
        cand = np.nonzero((fs == F_READ) & (typ == T_OK) & ~res_nil)[0]
        if len(cand):
            j = cand[rng.integers(0, len(cand))]
            res[j] = (res[j] + 1 + rng.integers(0, 4)) % 5
    zeros = np.zeros(n_ops, np.int64)
    # invocation values: read nil, write v, cas [old v]
    inv_vf = np.where(fs == F_READ, V_NIL, np.where(fs == F_WRITE, V_SCALAR, V_PAIR)).astype(np.int8)
    inv_a = np.where(fs == F_CAS, old, val)
    inv_b = np.where(fs == F_CAS, val, 0)
    # completion values: read -> observed (nil if absent); write/cas echo the invocation
    c_vf = np.where(fs == F_READ, np.where(res_nil, V_NIL, V_SCALAR), inv_vf).astype(np.int8)
    c_a = np.where(fs == F_READ, res, inv_a)
    c_b = np.where(fs == F_READ, zeros, inv_b)
    return _emit(n_clients, client, inv, cmp_, typ, fs, (inv_vf, inv_a, inv_b),
                 (c_vf, c_a, c_b), crashed)


def gen_counter(n_ops: int, n_clients: int, p_info: float, seed: int,
                invalid: bool = False, n_crashed: int | None = None,
                crash_span: float = 1.0) -> History:
    """n_crashed: exactly that many non-read ops time out (:info), drawn uniformly from the first
    `crash_span` of the ops (SURVEY §8(d) C5's exact-search variant, "<= ~15 crashed total");
    p_info then only makes reads :fail. Default (None): every non-read op crashes with
    probability p_info (the bounds-scan workload)."""
    rng = np.random.default_rng(seed)
    fs = np.array([F_READ, F_ADD, F_DECR, F_AAG, F_DAG], np.int8)[rng.integers(0, 5, n_ops)]
    d = rng.integers(0, 5, n_ops)
    crash_idx = None
    if n_crashed is not None:
        span = np.nonzero(fs[:max(1, int(n_ops * crash_span))] != F_READ)[0]
        crash_idx = np.random.default_rng(seed ^ 0xC5A5).choice(span, min(n_crashed, len(span)), replace=False)
    client, inv, cmp_, lin, crashed, read_fail, app_c = _schedule(rng, n_ops, n_clients, p_info, fs,
                                                                  crash_idx)
    typ = np.full(n_ops, T_OK, np.int8)
    res = np.zeros(n_ops, np.int64)
    state = 0
    sign = np.where((fs == F_DECR) | (fs == F_DAG), -1, 1)
    for i in np.argsort(lin, kind="stable"):
        f = fs[i]
        if f == F_READ:
            if read_fail[i]:
                typ[i] = T_FAIL
            else:
                res[i] = state
            continue
        if crashed[i]:
            typ[i] = T_INFO
            if not app_c[i]:
                continue
        state += int(sign[i] * d[i])
        res[i] = state
    if invalid:
        cand = np.nonzero((fs == F_READ) & (typ == T_OK))[0]
        if len(cand):
            j = cand[rng.integers(0, len(cand))]
            res[j] += 1 + rng.integers(0, 3)
    zeros = np.zeros(n_ops, np.int64)
    get = (fs == F_AAG) | (fs == F_DAG)
    inv_vf = np.where(fs == F_READ, V_NIL, V_SCALAR).astype(np.int8)
    inv_a = np.where(fs == F_READ, zeros, d)
    c_vf = np.where(fs == F_READ, V_SCALAR, np.where(get, V_PAIR, V_SCALAR)).astype(np.int8)
    c_a = np.where(fs == F_READ, res, d)
    c_b = np.where(get, res, zeros)
    return _emit(n_clients, client, inv, cmp_, typ, fs, (inv_vf, inv_a, zeros),
                 (c_vf, c_a, c_b), crashed)


def gen_leader(n_ops: int, n_clients: int, p_info: float, seed: int, invalid: bool = False,
               n_terms: int = 6, n_nodes: int = 5, p_crash: float = 0.0) -> History:
    """The :election workload (leader.clj:14-17, :38-40, :79-85): every op is :inspect, invoked
    with [nil 0] and completed with the [leader term] the cluster reports at its linearization
    point. Ground truth: term 0 without a leader ("null"), then terms 1..n_terms, each with one
    leader among n_nodes nodes ("n0".., interned ids), elections spread over the run. An
    inspect that times out is :fail (idempotent, client.clj:52-63), with probability p_info;
    p_crash > 0 also leaves ops :info (pending forever with their [nil 0] invoke value), to
    exercise the search's pending-op paths. invalid=True gives one :ok op of a term another
    :ok op also reports a different leader (a second leader in one term)."""
    rng = np.random.default_rng(seed)
    fs = np.full(n_ops, F_INSPECT, np.int8)
    client, inv, cmp_, lin, crashed, read_fail, _ = _schedule(rng, n_ops, n_clients, 0.0, fs)
    horizon = float(cmp_.max()) if n_ops else 1.0
    t_elect = np.sort(rng.uniform(0.0, horizon, n_terms))
    leaders = [leader_id(f"n{int(k)}") for k in rng.integers(0, n_nodes, n_terms)]
    term = np.searchsorted(t_elect, lin, side="right")  # 0 before the first election
    lead = np.array([leader_id(None)] + leaders, np.int64)[term]
    typ = np.full(n_ops, T_OK, np.int8)
    u = rng.uniform(size=n_ops)
    typ[u < p_info] = T_FAIL
    crashed = (u >= p_info) & (u < p_info + p_crash)
    typ[crashed] = T_INFO
    if invalid:
        ok = np.nonzero(typ == T_OK)[0]
        terms_ok = term[ok]
        multi = [i for i in ok if np.count_nonzero(terms_ok == term[i]) >= 2]
        if multi:
            j = multi[rng.integers(0, len(multi))]
            others = [leader_id(f"n{k}") for k in range(n_nodes) if leader_id(f"n{k}") != lead[j]]
            lead[j] = others[rng.integers(0, len(others))]
    zeros = np.zeros(n_ops, np.int64)
    pair = np.full(n_ops, V_PAIR, np.int8)
    inv_v = (pair, np.full(n_ops, leader_id(None), np.int64), zeros)  # [nil 0]
    cmp_v = (pair, lead.astype(np.int64), term.astype(np.int64))
    return _emit(n_clients, client, inv, cmp_, typ, fs, inv_v, cmp_v, crashed)


def gen_register_keys(n_keys: int, ops_per_key: int, n_clients: int, p_info: float,
                      config_id: int = 3, key0: int = 0, invalid_keys=()) -> History:
    """A jepsen.independent history, already split into per-key subhistories."""
    hs = []
    for k in range(key0, key0 + n_keys):
        h = gen_register(ops_per_key, n_clients, p_info, seed_for(config_id, k),
                         invalid=k in invalid_keys)
        h.keys = [k]
        hs.append(h)
    return concat(hs)


# BASELINE.json configs
CONFIGS = {
    "c1": dict(kind="register", n_keys=10, ops=200, clients=5, p_info=0.01),
    "c2": dict(kind="register", n_keys=1, ops=5000, clients=16, p_info=0.002),
    "c3": dict(kind="register", n_keys=1000, ops=1000, clients=5, p_info=0.01),
    "c4": dict(kind="register", n_keys=1, ops=100000, clients=16, p_info=1.5e-4),
    "c5": dict(kind="counter", n_keys=1, ops=1000000, clients=16, p_info=0.01),
    # counter histories for the exact search: c2c is C2's shape as a counter
    # (1 key x 5k ops, 16 clients, no crashes); c5x is C5's low-crash exact-search variant (SURVEY
    # §8(d): "exact search: <= ~15 crashed total"): 4 crashed ops in the first 1 % of the history,
    # so they stay pending (live) through all 1M ops; p_info 0.01 only fails reads
    "c2c": dict(kind="counter", n_keys=1, ops=5000, clients=16, p_info=0.0, seed=12345),
    "c5x": dict(kind="counter", n_keys=1, ops=1000000, clients=16, p_info=0.01, n_crashed=4,
                crash_span=0.01),
}


def gen_config(name: str, key0: int = 0, scale: float = 1.0) -> History:
    c = CONFIGS[name]
    cid = int(name[1])
    ops = max(1, int(c["ops"] * scale)) if c["n_keys"] == 1 else c["ops"]
    n_keys = c["n_keys"] if c["n_keys"] == 1 else max(1, int(c["n_keys"] * scale))
    if c["kind"] == "counter":
        h = gen_counter(ops, c["clients"], c["p_info"], c.get("seed", seed_for(cid, key0)),
                        n_crashed=c.get("n_crashed"), crash_span=c.get("crash_span", 1.0))
        h.keys = [key0]
        return h
    return gen_register_keys(n_keys, ops, c["clients"], c["p_info"], config_id=cid, key0=key0)


def perturb_read(h: History, at_frac: float, model: str = "cas-register", seed: int = 0) -> History:
    """A copy of single history h with ONE :ok read changed: the first :ok read completion at or
    after entry at_frac * n whose value is a scalar. A register read v becomes (v + 1 + r) % 5
    (another value of the generator's domain), a counter read v + 1 + r, r ~ U{0..3} from seed.
    The full-size invalid fixtures (tests/golden/pin_wide.py) stop the search mid-history."""
    from .history import from_columns
    t, f, vf = np.asarray(h.type), np.asarray(h.f), np.asarray(h.vflags)
    start = int(at_frac * h.n)
    cand = np.nonzero((t[start:] == T_OK) & (f[start:] == F_READ) & (vf[start:] == V_SCALAR))[0]
    if not len(cand):
        raise ValueError("no :ok scalar read after the requested point")
    j = start + int(cand[0])
    r = 1 + int(np.random.default_rng(seed).integers(0, 4))
    v0 = np.array(h.v0, copy=True)
    v0[j] = (v0[j] + r) % 5 if model == "cas-register" else v0[j] + r
    out = from_columns(np.array(h.index, copy=True), np.array(h.process, copy=True), t.copy(),
                       f.copy(), v0, np.array(h.v1, copy=True), vf.copy())
    out.keys = list(getattr(h, "keys", None) or [0])
    return out


def truncate(h: History, m: int) -> History:
    """Prefix of the first m entries of a single history (bounded CPU-baseline samples)."""
    from .history import from_columns
    return from_columns(h.index[:m], h.process[:m], h.type[:m], h.f[:m], h.v0[:m], h.v1[:m],
                        h.vflags[:m])
