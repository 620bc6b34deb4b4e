"""Independent checkers for small histories (test infrastructure).

* `brute_valid`: a Wing-Gong style exhaustive search over linearization orders (no JIT,
  no frontier) — decides linearizability of a history, optional :info ops included.
* `brute_first_failure`: the first :ok completion whose history prefix is not
  linearizable; the JIT search (knossos.linear [ext]) fails exactly there.
* `literal_search`: a literal restatement of the §8(a) contract with configs as
  (model value, frozenset of linearized op ids) — cross-checks explored/max_frontier.
Models follow knossos.model/CASRegister [ext] (register.clj:110), CounterModel
(counter.clj:100-127) and LeaderModel (leader.clj:63-75; state = frozenset of (term, leader)).
"""
from __future__ import annotations

from functools import lru_cache

NIL = ("nil",)


def _val(op):
    return op["value"]


def step(model, state, f, v):
    """Returns the next state or None if inconsistent."""
    if model == "leader":  # leader.clj:69-75 over a frozenset of (term, leader) pairs
        if f != "inspect":
            raise ValueError(f)
        leader, term = (v[0], v[1]) if v is not None else (None, None)
        name = "null" if leader is None else str(leader)
        for (t, l) in state:
            if t == term:
                return state if l == name else None
        return state | {(term, name)}
    if model == "cas-register":
        if f == "write":
            return NIL if v is None else v
        if f == "cas":
            cur, new = v
            return new if state == cur else None
        if f == "read":
            return state if (v is None or state == v) else None
        raise ValueError(f)
    if f == "add":
        return state + v
    if f == "decr":
        return state - v
    if f == "read":
        return state if (v is None or state == v) else None
    if f in ("add-and-get", "decr-and-get"):
        sg = 1 if f == "add-and-get" else -1
        if isinstance(v, (list, tuple)):
            d, new = v
            return new if state + sg * d == new else None
        return state + sg * v
    raise ValueError(f)


def preprocess(history):
    """Pair invocations with completions by process (knossos.history [ext]).
    Returns ops: dicts with inv, cmp (None if pending forever), f, value, ok."""
    pend, ops = {}, []
    for pos, o in enumerate(history):
        p = o["process"]
        if o["type"] == "invoke":
            rec = {"inv": pos, "cmp": None, "f": o["f"], "value": o["value"], "status": None,
                   "inv_index": o.get("index", pos)}
            pend[p] = rec
            ops.append(rec)
        else:
            rec = pend.pop(p)
            rec["status"] = o["type"]
            rec["cmp"] = pos
            rec["cmp_index"] = o.get("index", pos)
            if o["type"] == "ok":
                rec["value"] = o["value"]
    return [r for r in ops if r["status"] != "fail"]


def _init(model, init_value):
    return NIL if model == "cas-register" else frozenset() if model == "leader" else init_value


def brute_valid(model, history, init_value=0, upto=None):
    """Linearizable? If `upto` (a history position) is given, only the prefix history[:upto+1]
    is considered: ops completing later are open (optional)."""
    ops = preprocess(history)
    if upto is not None:
        ops = [o for o in ops if o["inv"] <= upto]
        req =[o["status"] == "ok" and o["cmp"] <= upto for o in ops]
    else:
        req = [o["status"] == "ok" for o in ops]
    n = len(ops)
    cmp_eff = [o["cmp"] if r else None for o, r in zip(ops, req)]
    required = frozenset(i for i in range(n) if req[i])

    def vfor(o):
        v = o["value"]
        return tuple(v) if isinstance(v, list) else v

    @lru_cache(maxsize=None)
    def go(done, state):
        if required <= done:
            return True
        for i in range(n):
            if i in done:
                continue
            # i may go next only if no not-yet-linearized required op completed before i's invoke
            if any(cmp_eff[j] is not None and cmp_eff[j] < ops[i]["inv"]
                   for j in range(n) if j not in done and j != i):
                continue
            s2 = step(model, state, ops[i]["f"], vfor(ops[i]))
            if s2 is None:
                continue
            if go(done | {i}, s2):
                return True
        return False

    return go(frozenset(), _init(model, init_value))


def brute_first_failure(model, history, init_value=0):
    """History position of the first :ok completion whose prefix is not linearizable."""
    for pos, o in enumerate(history):
        if o["type"] == "ok" and not brute_valid(model, history, init_value, upto=pos):
            return pos
    return -1


def literal_search(model, history, init_value=0):
    """The §8(a) contract, literally: configs are (state, frozenset(linearized op ids))."""
    ops = preprocess(history)
    by_inv = {o["inv"]: k for k, o in enumerate(ops)}
    by_cmp = {o["cmp"]: k for k, o in enumerate(ops) if o["status"] == "ok"}
    pending = []
    F = {(_init(model, init_value), frozenset())}
    explored, maxf, last_ok = 0, 1, -1

    def vfor(o):
        v = o["value"]
        return tuple(v) if isinstance(v, list) else v

    for pos, o in enumerate(history):
        if o["type"] == "invoke" and pos in by_inv:
            pending.append(by_inv[pos])
        elif o["type"] == "ok":
            t = by_cmp[pos]
            out, S = set(), set()
            level = []
            for (s, lin) in F:
                if t in lin:
                    out.add((s, lin - {t}))
                else:
                    level.append((s, lin))
            while level:
                nxt = []
                for (s, lin) in level:
                    for k in pending:
                        if k in lin:
                            continue
                        s2 = step(model, s, ops[k]["f"], vfor(ops[k]))
                        if s2 is None:
                            continue
                        c = (s2, lin | {k})
                        if c in S:
                            continue
                        S.add(c)
                        if k == t:
                            out.add((s2, lin))
                        else:
                            nxt.append(c)
                level = nxt
            explored += len(S)
            if not out:
                return {"valid": False, "fail_pos": pos, "explored": explored,
                        "max_frontier": maxf, "prev_ok_pos": last_ok, "frontier": F}
            F = out
            pending.remove(t)
            maxf = max(maxf, len(F))
            last_ok = pos
    return {"valid": True, "fail_pos": -1, "explored": explored, "max_frontier": maxf,
            "prev_ok_pos": -1, "frontier": F}


def literal_last_ops(model, history, init_value=0):
    """Knossos's per-config :last-op [ext], literally: the frontier carries (state, linearized
    set, last) triples for EVERY route (no dedup on `last`). A RETURN's closure stops where the
    returning op is linearized, so each config it emits has that op last; a config carried
    through a RETURN keeps its own. At the first failing :ok -> {(state, frozenset(invocation
    :index), sorted): set of the :ok completion :index values of every achievable last op (None: the
    initial config)}; None when the history is valid."""
    ops = preprocess(history)
    by_inv = {o["inv"]: k for k, o in enumerate(ops)}
    by_cmp = {o["cmp"]: k for k, o in enumerate(ops) if o["status"] == "ok"}
    pending = []
    F = {(_init(model, init_value), frozenset(), None)}

    def vfor(o):
        v = o["value"]
        return tuple(v) if isinstance(v, list) else v

    for pos, o in enumerate(history):
        if o["type"] == "invoke" and pos in by_inv:
            pending.append(by_inv[pos])
        elif o["type"] == "ok":
            t = by_cmp[pos]
            out, S, level = set(), set(), []
            for (s, lin, last) in F:
                if t in lin:
                    out.add((s, lin - {t}, last))
                elif (s, lin) not in S:
                    level.append((s, lin))
            while level:
                nxt = []
                for (s, lin) in level:
                    for k in pending:
                        if k in lin:
                            continue
                        s2 = step(model, s, ops[k]["f"], vfor(ops[k]))
                        if s2 is None or (s2, lin | {k}) in S:
                            continue
                        S.add((s2, lin | {k}))
                        if k == t:
                            out.add((s2, lin, ops[t]["cmp_index"]))
                        else:
                            nxt.append((s2, lin | {k}))
                level = nxt
            if not out:
                res = {}
                for (s, lin, last) in F:
                    key = (None if s == NIL else s, tuple(sorted(ops[k]["inv_index"] for k in lin)))
                    res.setdefault(key, set()).add(last)
                return res
            F = out
            pending.remove(t)
    return None
