"""lincheck — MI355X linearizability checker (drop-in for the reference's
checker/linearizable {:algorithm :linear} on cas-register and CounterModel histories)."""
from . import history, model
from .checker import (Checker, check_safe, compose, independent_checker, linearizable,
                      merge_valid, timeline_html)
from .model import CounterModel, LeaderModel, cas_register

__all__ = ["history", "model", "Checker", "check_safe", "compose", "independent_checker",
           "linearizable", "merge_valid", "timeline_html", "CounterModel", "LeaderModel", "cas_register"]
