"""Model descriptors mirroring the reference's models.

* cas_register()  -> knossos.model/cas-register [ext], used at register.clj:110
                     (initial value nil)
* CounterModel(v) -> jepsen.jgroups.workload.counter/CounterModel, counter.clj:100-127
                     (used as (CounterModel. 0), counter.clj:136)
* LeaderModel is out of scope (leader.clj:63-75: unbounded map state) — passing it
  raises, so a caller routes the :election workload to Knossos.
"""
from dataclasses import dataclass


@dataclass(frozen=True)
class Model:
    name: str
    kind: int
    init_value: int = 0


def cas_register(value=None) -> Model:
    if value is not None:
        raise ValueError("the GPU cas-register starts at nil, as (model/cas-register) does")
    return Model("cas-register", 1, 0)


def CounterModel(value: int = 0) -> Model:  # noqa: N802  (mirrors the Clojure record name)
    return Model("counter", 2, int(value))
