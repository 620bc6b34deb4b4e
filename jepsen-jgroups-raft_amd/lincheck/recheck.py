"""Offline re-check of a stored Jepsen history on the GPU.

    python -m lincheck.recheck store/<test>/<time>/history.edn --workload register
    python -m lincheck.recheck history.edn --workload counter --gpus 8

Reads the history with lincheck.edn and runs the same checker the reference's workload builds:
  register / single-register / multi-register:
      (independent/checker (checker/compose {:timeline .. :linear (checker/linearizable
          {:model (model/cas-register) :algorithm :linear})}))           register.clj:106-111
  counter:
      (checker/compose {:timeline .. :linear (checker/linearizable
          {:model (CounterModel. 0) :algorithm :linear})})                counter.clj:133-137
and prints the result map as JSON (keywords as strings, ops as maps).
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import Any, Dict, List

from . import checker as C
from .edn import read_history
from .history import KV
from .model import CounterModel, cas_register

WORKLOADS = ("register", "single-register", "multi-register", "counter")


def workload_checker(workload: str, gpus: int = 1) -> C.Checker:
    if workload in ("register", "single-register", "multi-register"):
        return C.independent_checker(C.compose({
            "timeline": C.timeline_html(),
            "linear": C.linearizable({"model": cas_register(), "algorithm": "linear",
                                      "gpus": gpus})}))
    if workload == "counter":
        return C.compose({
            "timeline": C.timeline_html(),
            "linear": C.linearizable({"model": CounterModel(0), "algorithm": "linear",
                                      "gpus": gpus})})
    raise ValueError(f"unknown workload {workload!r} (one of {', '.join(WORKLOADS)}; "
                     "the election workload's LeaderModel stays on Knossos)")


def recheck(ops: List[Dict[str, Any]], workload: str, gpus: int = 1) -> Dict[str, Any]:
    return C.check_safe(workload_checker(workload, gpus), {"name": "recheck"}, ops, {})


def _jsonable(x):
    if isinstance(x, KV):
        return [_jsonable(x.key), _jsonable(x.value)]
    if isinstance(x, dict):
        return {str(k): _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple, set, frozenset)):
        return [_jsonable(v) for v in x]
    return x


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("history", help="history.edn (one op map per line, or a vector of ops)")
    ap.add_argument("--workload", required=True, choices=WORKLOADS)
    ap.add_argument("--gpus", type=int, default=1)
    args = ap.parse_args(argv)
    independent = args.workload != "counter"
    ops = read_history(args.history, independent=independent)
    res = recheck(ops, args.workload, args.gpus)
    print(json.dumps(_jsonable(res), default=str))
    return 0 if res.get("valid?") is True else 1


if __name__ == "__main__":
    sys.exit(main())
