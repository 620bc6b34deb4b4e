"""Model descriptors mirroring the reference's models.

* cas_register()  -> knossos.model/cas-register [ext], used at register.clj:110
                     (initial value nil)
* CounterModel(v) -> jepsen.jgroups.workload.counter/CounterModel, counter.clj:100-127
                     (used as (CounterModel. 0), counter.clj:136)
* LeaderModel()   -> jepsen.jgroups.workload.leader/LeaderModel, leader.clj:63-75 (used as
                     (LeaderModel. {}), leader.clj:84). Out of the GPU's scope (unbounded
                     term -> leader map state): linearizable() returns
                     the fallback map, and the JVM binding hands it to Knossos unchanged.
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
    return Model("leader", 0, 0, gpu=False)
