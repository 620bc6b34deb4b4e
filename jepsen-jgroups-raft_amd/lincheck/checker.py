"""jepsen.checker-shaped host API over liblincheck.so.

Mirrors the reference's call sites:
  (checker/linearizable {:model (model/cas-register) :algorithm :linear})   register.clj:109-111
  (checker/linearizable {:model (CounterModel. 0) :algorithm :linear})      counter.clj:135-137
  (independent/checker (checker/compose {:timeline .. :linear ..}))         register.clj:106-111
A Checker's check(test, history, opts) returns the Knossos-keyed map: "valid?" (True, False
or "unknown"), "analyzer", and on failure "op", "previous-ok", "last-op", "configs" (<= 10,
compare as a set), plus "explored" (SURVEY §8(a) contract). Errors raised by the native
layer propagate, as they would out of Knossos; jepsen's check-safe [ext] turns them into
{:valid? :unknown :error ...}, which `check_safe` below mirrors.
"""
from __future__ import annotations

import traceback
from typing import Any, Dict, List, Optional, Sequence

from . import _lib
from . import history as H
from .model import Inconsistent, Model, step

VALID = {1: True, 0: False, 2: "unknown"}
ERRORS = {0: None, -4: "malformed history", -5: "too many concurrently pending ops",
          -6: "model cannot step an op", -7: "frontier exceeded max-configs / device capacity",
          -8: "device search aborted by its barrier watchdog (device not wholly available)"}


def merge_valid(vs: Sequence[Any]):
    """jepsen.checker/merge-valid [ext]: false beats :unknown beats true."""
    vs = list(vs)
    if any(v is False for v in vs):
        return False
    if any(v == "unknown" for v in vs):
        return "unknown"
    return True


class Checker:
    def check(self, test, history, opts=None) -> Dict[str, Any]:
        raise NotImplementedError


def _op_at(ops: List[Dict[str, Any]], index: int) -> Optional[Dict[str, Any]]:
    if index < 0:
        return None
    for o in ops:
        if o.get("index") == index:
            return o
    return ops[index] if 0 <= index < len(ops) else None


def _folded_ops(ops) -> Dict[int, Dict[str, Any]]:
    """invocation :index -> the op as the model steps it (knossos.history/complete [ext]: an
    :ok completion's value folded into its invocation; :info keeps the invocation's)."""
    by_proc: Dict[Any, Dict[str, Any]] = {}
    out: Dict[int, Dict[str, Any]] = {}
    for pos, o in enumerate(ops):
        t = str(o.get("type", "")).lstrip(":")
        idx = int(o.get("index", pos))
        if t == "invoke":
            op = {"index": idx, "process": o.get("process"), "f": str(o["f"]).lstrip(":"),
                  "value": o.get("value")}
            by_proc[o.get("process")] = op
            out[idx] = op
        elif o.get("process") in by_proc:
            op = by_proc.pop(o.get("process"))
            if t == "ok":
                op["value"] = o.get("value")
    return out


def final_paths(model: Model, configs, pending, fail_inv: int, ops, k: int = 10):
    """:final-paths of a Knossos failure report [ext] (jepsen.checker/linearizable keeps <= 10):
    from each pre-failure config, sequences of pending ops linearized one after another, each
    step consistent, ending with the failing op, whose step is inconsistent. Every config the
    search reaches fails that op (that is why the verdict is false), so each path ends there.
    Breadth-first (shortest paths first), pending ops in :index order. Each path is a list of
    {"op", "model"}: the config's value first (op None), then every op with the value after it;
    the last model is {"inconsistent": message}."""
    folded = _folded_ops(ops)
    fop = folded.get(fail_inv)
    if fop is None:
        return []
    order = sorted(pending)
    paths = []
    queue = [((None if s is None else s) if model.name in ("cas-register", "leader") else (s or 0),
              frozenset(lin), [{"op": None, "model": {"value": s}}]) for (s, lin) in configs]
    while queue and len(paths) < k:
        nxt = []
        for value, lin, path in queue:
            r = step(model, value, fop["f"], fop["value"])
            if isinstance(r, Inconsistent):
                paths.append(path + [{"op": fop, "model": {"inconsistent": str(r)}}])
                if len(paths) >= k:
                    break
            for i in order:
                if i in lin or i == fail_inv or i not in folded:
                    continue
                o = folded[i]
                r2 = step(model, value, o["f"], o["value"])
                if not isinstance(r2, Inconsistent):
                    nxt.append((r2, lin | {i}, path + [{"op": o, "model": {"value": r2}}]))
        queue = nxt
    return paths


def _leader_maps(ops, fail_idx: int, cfgs):
    """LeaderModel configs: the device reports each config's contested pairs only, so its
    term -> leader map is rebuilt as the search defines it: the (term, leader) pairs of every
    op that returned :ok before the failing completion, plus the pending ops the config has
    linearized (leader.clj:69-75: a consistent map has one leader per term)."""
    folded = _folded_ops(ops)
    returned, by_proc = [], {}
    for pos, o in enumerate(ops):
        idx = int(o.get("index", pos))
        if idx == fail_idx:
            break
        t = str(o.get("type", "")).lstrip(":")
        if t == "invoke":
            by_proc[o.get("process")] = idx
        elif o.get("process") in by_proc:
            inv = by_proc.pop(o.get("process"))
            if t == "ok":
                returned.append(inv)
    out = []
    for _s, lin in cfgs:
        state = None
        for i in returned + sorted(lin):
            fo = folded.get(i)
            if fo is not None:
                state = step(Model("leader", 3), state, "inspect", fo["value"])
        out.append((state or {}, lin))
    return out


def _result_map(ops, r, k, model: Model, configs=None) -> Dict[str, Any]:
    v = VALID[int(r["valid"][k])]
    out: Dict[str, Any] = {"valid?": v, "analyzer": "linear",
                           "explored": int(r["explored"][k])}
    err = ERRORS.get(int(r["err"][k]))
    if err:
        out["error"] = err
    if v is False:
        out["op"] = _op_at(ops, int(r["fail_idx"][k]))
        out["previous-ok"] = _op_at(ops, int(r["prev_ok"][k]))
        out["invocation"] = _op_at(ops, int(r["fail_inv"][k]))
        # :last-op: the op linearized last on the way to the pre-failure frontier, from the
        # search (lc_failure_configs: each config's own, the newest over the frontier here).
        # Without a report it is :previous-ok's op: a RETURN's closure stops where the
        # returning op is linearized, so every config the previous RETURN emitted has it last.
        out["last-op"] = out["previous-ok"]
        if configs is not None:
            cfgs, pending, lasts, newest = configs
            if model.name == "leader":
                cfgs = _leader_maps(ops, int(r["fail_idx"][k]), cfgs)
            out["last-op"] = _op_at(ops, newest)
            # Knossos :configs [ext]: {:model :last-op :pending}, :pending = the calls this
            # config has not linearized (invocations, :index order)
            out["configs"] = [{"model": {"value": s}, "last-op": _op_at(ops, last),
                               "pending": [_op_at(ops, i) for i in sorted(pending) if i not in lin]}
                              for (s, lin), last in zip(cfgs, lasts)]
            out["final-paths"] = final_paths(model, cfgs, pending, int(r["fail_inv"][k]), ops)
    return out


class Linearizable(Checker):
    """(checker/linearizable {:model m :algorithm :linear}) on the GPU."""

    def __init__(self, opts: Dict[str, Any]):
        m = opts.get("model")
        if not isinstance(m, Model):
            raise ValueError("model must be lincheck.model.cas_register(), CounterModel(v) or "
                             "LeaderModel()")
        alg = opts.get("algorithm", "linear")
        if str(alg).lstrip(":") not in ("linear", "competition", "wgl"):
            raise ValueError(f"unknown algorithm {alg!r}")
        self.model = m
        self.n_gpus = int(opts.get("gpus", 1))
        self.max_configs = int(opts.get("max-configs", 0))
        self.report_configs = bool(opts.get("configs", True))

    def check_many(self, h: H.History, ops_per_hist=None) -> List[Dict[str, Any]]:
        if not self.model.gpu:
            return [fallback_result(self.model) for _ in range(h.n_hist)]
        r = _lib.check(self.model.kind, self.model.init_value, h, self.n_gpus, self.max_configs)
        outs = []
        for k in range(h.n_hist):
            ops = ops_per_hist[k] if ops_per_hist is not None else h.to_ops(k)
            cfg = None
            cfg_err = None
            if self.report_configs and r["valid"][k] == 0:
                # the report is extra: if the frontier dump fails, the verdict still stands
                try:
                    cfg = _lib.failure_configs(k, 10, with_last=True)
                except _lib.LincheckError as e:
                    cfg_err = str(e)
            res = _result_map(ops, r, k, self.model, cfg)
            if cfg_err is not None:
                res["configs-error"] = cfg_err
            outs.append(res)
        return outs

    def check(self, test, history, opts=None) -> Dict[str, Any]:
        if not self.model.gpu:
            return fallback_result(self.model)
        ops = [o for o in history if H.client_op(o)]
        h = H.encode(ops)
        return self.check_many(h, [h.to_ops(0)])[0] if h.n else \
            {"valid?": True, "analyzer": "linear", "explored": 0}


def fallback_result(model: Model) -> Dict[str, Any]:
    """The map a model the GPU search does not implement gets (a Model(gpu=False); every model
    the suite uses, LeaderModel included since r3, is searched on the GPU): the JVM binding
    routes such a model to knossos.linear/analysis unchanged. This host
    mirror has no Knossos to route to and reports the hand-off as :unknown, the shape jepsen's
    check-safe gives a checker that cannot decide [ext]."""
    return {"valid?": "unknown", "analyzer": "linear", "fallback": "knossos",
            "error": f"model {model.name} is not searched on the GPU: route it to "
                     "knossos.linear/analysis (the JVM binding's fallback)"}


def linearizable(opts: Dict[str, Any]) -> Linearizable:
    return Linearizable(opts)


class Compose(Checker):
    """jepsen.checker/compose [ext]: run each checker, merge :valid?."""

    def __init__(self, checkers: Dict[str, Checker]):
        self.checkers = checkers

    def check(self, test, history, opts=None):
        res = {k: c.check(test, history, opts) for k, c in self.checkers.items()}
        res["valid?"] = merge_valid(r["valid?"] for r in res.values())
        return res


def compose(checkers: Dict[str, Checker]) -> Compose:
    return Compose(checkers)


class Independent(Checker):
    """jepsen.independent/checker [ext] (register.clj:106): split by key, check every key.
    All keys whose inner checker is a Linearizable go down in ONE lc_check call (the GPU
    batches them); results come back as {"valid?", "results": {k: r}, "failures": [k ...]}."""

    def __init__(self, inner: Checker):
        self.inner = inner

    def _lin(self) -> Optional[Linearizable]:
        if isinstance(self.inner, Linearizable):
            return self.inner
        if isinstance(self.inner, Compose):
            lins = [c for c in self.inner.checkers.values() if isinstance(c, Linearizable)]
            return lins[0] if len(lins) == 1 else None
        return None

    def check(self, test, history, opts=None):
        h = H.subhistories(history)
        lin = self._lin()
        results: Dict[Any, Dict[str, Any]] = {}
        if lin is not None and h.n_hist:
            rs = lin.check_many(h)
            for k, key in enumerate(h.keys):
                if isinstance(self.inner, Compose):
                    name = [n for n, c in self.inner.checkers.items() if c is lin][0]
                    r = {name: rs[k]}
                    for n, c in self.inner.checkers.items():
                        if c is not lin:
                            r[n] = c.check(test, h.to_ops(k), opts)
                    r["valid?"] = merge_valid(x["valid?"] for x in r.values())
                else:
                    r = rs[k]
                results[key] = r
        else:
            for k, key in enumerate(h.keys or []):
                results[key] = self.inner.check(test, h.to_ops(k), opts)
        # jepsen.independent/checker [ext]: keys whose :valid? is falsey (:unknown is truthy)
        failures = [k for k, r in results.items() if r["valid?"] is False]
        return {"valid?": merge_valid(r["valid?"] for r in results.values()) if results else True,
                "results": results, "failures": failures}


def independent_checker(inner: Checker) -> Independent:
    return Independent(inner)


def check_safe(checker: Checker, test, history, opts=None):
    """jepsen.checker/check-safe [ext]: exceptions become {:valid? :unknown :error ...}."""
    try:
        return checker.check(test, history, opts)
    except Exception as e:  # noqa: BLE001 — mirrors check-safe's catch-all
        return {"valid?": "unknown", "error": "".join(traceback.format_exception_only(type(e), e))}


class Noop(Checker):
    """Stand-in for (timeline/html): rendering is out of scope; always valid."""

    def check(self, test, history, opts=None):
        return {"valid?": True}


def timeline_html() -> Noop:
    return Noop()
