"""Model descriptors mirroring the reference's models.

* cas_register()  -> knossos.model/cas-register [ext], used at register.clj:110
                     (initial value nil)
* CounterModel(v) -> jepsen.jgroups.workload.counter/CounterModel, counter.clj:100-127
                     (used as (CounterModel. 0), counter.clj:136)
* LeaderModel()   -> jepsen.jgroups.workload.leader/LeaderModel, leader.clj:63-75 (used as
                     (LeaderModel. {}), leader.clj:84; the :election workload). The GPU search
                     keeps its term -> leader map as the set of linearized (term, leader) pairs
                     of the terms that carry two or more leaders (include/lincheck.h).
"""
from dataclasses import dataclass


@dataclass(frozen=True)
class Model:
    name: str
    kind: int
    init_value: int = 0
    gpu: bool = True  # False: routed to the Knossos fallback (checker.fallback_result)


def cas_register(value=None) -> Model:
    if value is not None:
        raise ValueError("the GPU cas-register starts at nil, as (model/cas-register) does")
    return Model("cas-register", 1, 0)


def CounterModel(value: int = 0) -> Model:  # noqa: N802  (mirrors the Clojure record name)
    return Model("counter", 2, int(value))


def LeaderModel(state=None) -> Model:  # noqa: N802  (mirrors the Clojure record name)
    if state:
        raise ValueError("LeaderModel starts from the empty term map, as (LeaderModel. {}) does")
    return Model("leader", 3, 0)


def serialize_leader(addr) -> str:
    """leader.clj:51-54: nil -> "null", else the name."""
    return "null" if addr is None else str(addr)


class Inconsistent(str):
    """knossos.model/inconsistent [ext]: a step the model cannot take (its message)."""


def step(model: Model, value, f: str, v):
    """One model step on a plain value, for failure reports (the search itself runs on the
    GPU). cas-register (knossos.model/CASRegister [ext]; register.clj:110): write v -> v;
    cas [cur new] -> new iff cur = value; read v -> value iff v is nil or v = value.
    CounterModel (counter.clj:100-127): add d -> value + d; decr d -> value - d; read x ->
    value iff x nil or x = value; add-and-get [d n] -> n iff value + d = n (scalar d, the
    :info case: value + d); decr-and-get mirrors it with -. LeaderModel (leader.clj:69-75):
    inspect [l t] -> the map with t -> l, inconsistent when it holds t with another leader.
    Returns the new value or an Inconsistent message."""
    if model.name == "cas-register":
        if f == "write":
            return v
        if f == "cas":
            cur, new = v
            return new if cur == value else Inconsistent(f"can't CAS {value} from {cur} to {new}")
        if f == "read":
            return value if v is None or v == value else Inconsistent(f"can't read {v} from register {value}")
    elif model.name == "counter":
        if f in ("add", "decr"):
            return value + v if f == "add" else value - v
        if f == "read":
            return value if v is None or v == value else Inconsistent(f"can't read {v} from counter {value}")
        if f in ("add-and-get", "decr-and-get"):
            sign = 1 if f == "add-and-get" else -1
            if isinstance(v, (list, tuple)):
                d, n = v
                return n if value + sign * d == n else Inconsistent(
                    f"{'adding' if sign > 0 else 'decreasing'} {d} to {value} should result in {n}")
            return value + sign * v
    elif model.name == "leader":
        # LeaderModel.step (leader.clj:69-75) on the term -> leader map (None: {})
        if f == "inspect":
            state = dict(value or {})
            inspected, t = (v[0], v[1]) if v is not None else (None, None)
            l = serialize_leader(inspected)
            if t in state and state[t] != l:
                return Inconsistent(f"leader at {t} was {state[t]} but received {l}")
            state[t] = l
            return state
    return Inconsistent(f"unknown :f {f} for {model.name}")
