"""CPU-side tests: the C-ABI library loads and exports every declared symbol, fails loudly
without a device, and the host-side Python mirror (encoding, independent split, merge-valid,
synthetic generator) behaves like the reference's."""
import os
import re

import numpy as np
import pytest

import oracle
from lincheck import _lib, checker, history as H, model, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "lincheck.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|void)\s+(lc_\w+)\s*\(", hdr, re.M)))


def test_header_matches_binding():
    assert _declared() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    L = _lib.load()
    for s in _declared():
        assert hasattr(L, s), s
    assert L.lc_abi_version() == 1


def test_no_device_fails_loudly():
    L = _lib.load()
    if L.lc_device_count() > 0:
        pytest.skip("a GPU is visible")
    h = synth.gen_register(10, 2, 0.0, 1)
    with pytest.raises(_lib.LincheckError, match="no HIP device"):
        _lib.check(1, 0, h)
    with pytest.raises(_lib.LincheckError):
        _lib.counter_bounds(0, synth.gen_counter(10, 2, 0.0, 1))
    with pytest.raises(_lib.LincheckError):
        _lib.Plan(1, 0, h)


def test_encode_roundtrip_and_client_filter():
    ops = [{"process": 0, "type": "invoke", "f": "cas", "value": [1, 2], "index": 0},
           {"process": "nemesis", "type": "info", "f": "start", "value": None, "index": 1},
           {"process": 0, "type": "ok", "f": "cas", "value": [1, 2], "index": 2},
           {"process": 1, "type": ":invoke", "f": ":read", "value": None, "index": 3}]
    h = H.encode(ops)
    assert h.n == 3
    back = h.to_ops()
    assert [o["index"] for o in back] == [0, 2, 3]
    assert back[0]["value"] == [1, 2] and back[2]["value"] is None


def test_subhistories_split_by_key():
    ops = []
    for i in range(6):
        k = i % 2
        ops.append({"process": i, "type": "invoke", "f": "write", "value": H.tuple_(k, i)})
        ops.append({"process": i, "type": "ok", "f": "write", "value": H.tuple_(k, i)})
    ops.append({"process": "nemesis", "type": "info", "f": "kill", "value": None})
    h = H.subhistories(ops)
    assert h.keys == [0, 1] and h.n_hist == 2 and h.n == 12
    assert list(h.sub(1).index) == [2, 3, 6, 7, 10, 11]
    assert all(isinstance(o["value"], int) for o in h.to_ops(0))


def test_merge_valid():
    assert checker.merge_valid([True, True]) is True
    assert checker.merge_valid([True, "unknown"]) == "unknown"
    assert checker.merge_valid(["unknown", False, True]) is False


def test_models_mirror_reference():
    assert model.cas_register().kind == 1
    assert model.CounterModel(0).init_value == 0
    with pytest.raises(ValueError):
        model.cas_register(3)
    with pytest.raises(ValueError):
        checker.linearizable({"model": "leader"})


def test_check_safe_turns_errors_into_unknown():
    class Boom(checker.Checker):
        def check(self, test, history, opts=None):
            raise RuntimeError("boom")
    r = checker.check_safe(Boom(), {}, [])
    assert r["valid?"] == "unknown" and "boom" in r["error"]


@pytest.mark.parametrize("gen,model_name", [(synth.gen_register, "cas-register"),
                                            (synth.gen_counter, "counter")])
def test_synthetic_histories_are_linearizable(gen, model_name):
    """The simulated SUT is linearizable by construction."""
    for s in range(20):
        h = gen(150, 5, 0.02, 100 + s)
        assert oracle.check_one(model_name, h)["valid"] == 1


def test_synthetic_invalid_variant_is_caught_sometimes():
    bad = sum(oracle.check_one("cas-register", synth.gen_register(200, 3, 0.0, 700 + s,
                                                                   invalid=True))["valid"] == 0
              for s in range(20))
    assert bad >= 10


def test_synth_shapes_follow_reference_domains():
    h = synth.gen_register(3000, 5, 0.05, 3)
    assert set(np.unique(h.f)) <= {0, 1, 2}
    inv = h.type == 0
    assert h.v0[inv & (h.f == 1)].max() <= 4 and h.v0[inv & (h.f == 1)].min() >= 0
    # reads never :info (idempotent, client.clj:59-62); cas failures are :fail
    reads = h.f == 0
    assert not np.any(reads & (h.type == 3))
    # a process has at most one outstanding op
    pend = {}
    for t, p in zip(h.type, h.process):
        if t == 0:
            assert not pend.get(p)
            pend[p] = True
        else:
            pend[p] = False


def test_seeds_follow_survey():
    assert synth.seed_for(3, 7) == 0x5EED0000 + 3007
