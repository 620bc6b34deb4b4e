"""Oracle pinning: the reference's golden vectors, hand KATs, and two independent
restatements (brute-force linearization search, literal frozenset search)."""
import json
import sys
import os
import random

import numpy as np
import pytest

import oracle
from brute import brute_first_failure, brute_valid, literal_last_ops, literal_search
from lincheck import history as H
from lincheck import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kats.json")
KATS = json.load(open(GOLD))


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_oracle_kats(kat):
    h = H.encode(kat["history"])
    r = oracle.check_one(kat["model"], h)
    assert r["valid"] == (1 if kat["valid"] else 0), r
    assert r["fail_idx"] == kat["fail_idx"]
    if kat["prev_ok_idx"] is not None:
        assert r["prev_ok_idx"] == kat["prev_ok_idx"]
    if kat["explored"] is not None:
        assert r["explored"] == kat["explored"], r


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_brute_agrees_with_kats(kat):
    assert brute_valid(kat["model"], kat["history"]) == kat["valid"]
    lit = literal_search(kat["model"], kat["history"])
    assert lit["valid"] == kat["valid"]
    if kat["explored"] is not None:
        assert lit["explored"] == kat["explored"]


def _small_random(model, seed, n_ops, clients, p_info, invalid):
    if model == "leader":
        return synth.gen_leader(n_ops, clients, p_info, seed, invalid=invalid, n_terms=2,
                                n_nodes=3, p_crash=0.25)
    g = synth.gen_register if model == "cas-register" else synth.gen_counter
    return g(n_ops, clients, p_info, seed, invalid=invalid)


@pytest.mark.parametrize("model", ["cas-register", "counter", "leader"])
def test_oracle_vs_brute_random(model):
    rng = random.Random(7)
    checked = 0
    for t in range(120):
        n_ops = rng.randint(1, 7)
        h = _small_random(model, 1000 + t, n_ops, rng.randint(1, 4), 0.3, invalid=(t % 2 == 1))
        ops = h.to_ops()
        r = oracle.check_one(model, h)
        exp_valid = brute_valid(model, ops)
        assert r["valid"] == (1 if exp_valid else 0), (ops, r)
        ff = brute_first_failure(model, ops)
        assert r["fail_idx"] == (ff if ff < 0 else int(h.index[ff])), (ops, r)
        lit = literal_search(model, ops)
        assert lit["explored"] == r["explored"], (ops, r, lit)
        assert lit["max_frontier"] == r["max_frontier"]
        checked += 1
    assert checked == 120


@pytest.mark.parametrize("model", ["cas-register", "counter", "leader"])
def test_oracle_vs_literal_medium(model):
    """Larger random histories (no brute force): the literal restatement must agree on
    verdict, failing index, explored count and max frontier."""
    for t in range(12):
        if model == "leader":
            h = synth.gen_leader(60, 4, 0.05, 5000 + t, invalid=(t % 3 == 2), p_crash=0.05)
        else:
            g = synth.gen_register if model == "cas-register" else synth.gen_counter
            h = g(60, 4, 0.05, 5000 + t, invalid=(t % 3 == 2))
        ops = h.to_ops()
        r = oracle.check_one(model, h)
        lit = literal_search(model, ops)
        assert r["valid"] == (1 if lit["valid"] else 0)
        assert r["fail_idx"] == lit["fail_pos"]
        assert r["explored"] == lit["explored"]
        assert r["max_frontier"] == lit["max_frontier"]


def test_oracle_failure_configs_match_literal():
    for t in range(40):
        h = synth.gen_register(40, 4, 0.1, 9000 + t, invalid=True)
        ops = h.to_ops()
        r = oracle.check_one("cas-register", h, with_configs=True)
        lit = literal_search("cas-register", ops)
        if not lit["valid"]:
            exp = set()
            pre = H.from_columns([], [], [], [], [], [], [])
            for (s, lin) in lit["frontier"]:
                inv_idx = tuple(sorted(ops[_inv_pos(ops, k)]["index"] for k in lin))
                exp.add((None if s == ("nil",) else s, inv_idx))
            assert r["fail_configs"] == exp


def _inv_pos(ops, k):
    # k is the op ordinal in brute.preprocess order (non-failed invocations)
    from brute import preprocess
    return preprocess(ops)[k]["inv"]


def test_errors_are_unknown():
    # completion without invocation
    h = H.encode([{"process": 0, "type": "ok", "f": "read", "value": 1}])
    assert oracle.check_one("cas-register", h)["valid"] == 2
    # unknown :f for the counter model (condp throws, counter.clj:102)
    h = H.encode([{"process": 0, "type": "invoke", "f": "write", "value": 1},
                  {"process": 0, "type": "ok", "f": "write", "value": 1}])
    assert oracle.check_one("counter", h)["valid"] == 2
    # max_configs exceeded -> unknown
    h = synth.gen_register(200, 8, 0.2, 77)
    assert oracle.check_one("cas-register", h, max_configs=1)["valid"] == 2


def test_check_many_matches_single():
    h = synth.gen_register_keys(16, 100, 5, 0.02, config_id=1)
    many = oracle.check_many("cas-register", h, n_threads=4)
    for k in range(h.n_hist):
        one = oracle.check_one("cas-register", h.sub(k))
        assert many[k].pop("wall_ns") > 0 and one.pop("wall_ns") == 0
        assert many[k] == one


def test_counter_bounds_sound():
    """The bounds filter never rejects a linearizable history and agrees with brute force
    whenever it rejects."""
    rejected = 0
    for t in range(200):
        h = synth.gen_counter(8, 3, 0.2, 300 + t, invalid=(t % 2 == 1))
        ok, bad = oracle.counter_bounds(h)
        lin = brute_valid("counter", h.to_ops())
        if lin:
            assert ok
        if not ok:
            rejected += 1
            assert not lin
    assert rejected > 10


@pytest.mark.parametrize("model", ["cas-register", "counter"])
def test_oracle_failure_last_ops_vs_literal(model):
    """Per-config :last-op of the failure report (Knossos's :configs [ext]): the oracle keeps,
    per pre-failure config, the most recent op it can have linearized last. Checked against a
    literal search that carries every route's last op: the oracle's is achievable and is the
    latest of them. Parity vs Knossos itself is unpinned (no Knossos here)."""
    n_cfg = n_multi = 0
    for t in range(200):
        g = synth.gen_register if model == "cas-register" else synth.gen_counter
        h = g(30, 4, 0.15, 7000 + t, invalid=True)
        r = oracle.check_one(model, h, with_configs=True)
        if r["valid"] != 0:
            continue
        lit = literal_last_ops(model, h.to_ops())
        assert set(lit) == r["fail_configs"]
        for c, lasts in lit.items():
            want = max(-1 if x is None else x for x in lasts)
            assert r["fail_last_op"][c] == want, (t, c, lasts, r["fail_last_op"][c])
            n_cfg += 1
            n_multi += len(lasts) > 1
    assert n_cfg > 50 and n_multi > 0, (n_cfg, n_multi)


def test_leader_model_step_literal():
    """LeaderModel.step (leader.clj:69-75) on literal maps: the empty map takes any term; a held
    term keeps the map for its own leader and is inconsistent for another; nil leaders
    serialize to "null" (leader.clj:51-54), so [nil t] and ["null" t] agree."""
    from lincheck import model as M
    L = M.LeaderModel()
    s = M.step(L, None, "inspect", ["n1", 3])
    assert s == {3: "n1"}
    assert M.step(L, s, "inspect", ["n1", 3]) == {3: "n1"}
    assert isinstance(M.step(L, s, "inspect", ["n2", 3]), M.Inconsistent)
    assert "leader at 3 was n1 but received n2" == str(M.step(L, s, "inspect", ["n2", 3]))
    assert M.step(L, s, "inspect", [None, 4]) == {3: "n1", 4: "null"}
    assert M.step(L, {4: "null"}, "inspect", ["null", 4]) == {4: "null"}
    assert M.step(L, {}, "inspect", None) == {None: "null"}


def test_leader_encoding_round_trip():
    """:inspect values encode as (leader id, term) pairs, nil and "null" to one id, and decode
    back to names."""
    ops = [{"process": 0, "type": "invoke", "f": "inspect", "value": [None, 0]},
           {"process": 0, "type": "ok", "f": "inspect", "value": ["n1", 2, "extra"]},
           {"process": 1, "type": "invoke", "f": "inspect", "value": [None, 0]},
           {"process": 1, "type": "ok", "f": "inspect", "value": ["null", 2]}]
    h = H.encode(ops)
    assert list(h.f) == [7] * 4 and list(h.vflags) == [2] * 4
    assert h.v0[0] == h.v0[2] == h.v0[3] == -1 and h.v0[1] >= 0 and list(h.v1) == [0, 2, 0, 2]
    back = h.to_ops()
    assert back[1]["value"] == ["n1", 2] and back[3]["value"] == [None, 2]
    r = oracle.check_one("leader", h)  # (2, n1) and (2, null): a second leader for term 2
    assert r["valid"] == 0 and r["fail_idx"] == 3 and brute_valid("leader", ops) is False


def test_leader_oracle_failure_configs_vs_literal():
    """Failure report configs and per-config :last-op for LeaderModel histories, against the
    literal search (its states are term maps, the oracle's pair bitmasks; a config's state is a
    function of its linearized set, so configs compare by that set)."""
    n = 0
    for t in range(120):
        h = synth.gen_leader(30, 4, 0.1, 8800 + t, invalid=True, n_terms=3, p_crash=0.15)
        r = oracle.check_one("leader", h, with_configs=True)
        if r["valid"] != 0:
            continue
        lit = literal_last_ops("leader", h.to_ops())
        got = {lin: r["fail_last_op"][(s, lin)] for (s, lin) in r["fail_configs"]}
        want = {lin: max(-1 if x is None else x for x in lasts) for (_s, lin), lasts in lit.items()}
        assert got == want, t
        n += 1
    assert n > 40


def test_c4_fixture_matches_generator():
    """tests/golden/c4_oracle.json (the full-size C4 oracle run, tests/golden/pin_c4.py) was
    made from this generator's C4 history: same entry and op counts, and its first 4k entries
    check the same way here (the GPU suite compares every path's explored count with it)."""
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "c4_oracle.json")))
    h = synth.gen_config("c4")
    assert (h.n, h.n_ops()) == (gold["n_entries"], gold["n_ops"])
    assert gold["valid"] == 1 and gold["explored"] == 10_994_841_001
    r = oracle.check_one("cas-register", synth.truncate(h, 4000))
    assert r["valid"] == 1 and r["explored"] > 0


@pytest.mark.parametrize("name", ["c2c", "c2c4", "c5x"])
def test_counter_fixtures_match_generator(name):
    """tests/golden/counter_<name>_oracle.json (the oracle's whole-history counter search at size,
    tests/golden/pin_counter.py) was made from this generator's history: same entry and op
    counts and the same column digest; c2c (5 s on one core) is re-checked here in full."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import pin_counter
    p = pin_counter.path_of(name)
    if not os.path.exists(p):
        pytest.skip(f"{name} not pinned yet")
    gold = json.load(open(p))
    h = pin_counter.GEN[name][1]()
    assert (h.n, h.n_ops()) == (gold["n_entries"], gold["n_ops"])
    assert pin_counter.digest(h) == gold["digest"]
    assert gold["err_code"] == 0 and gold["valid"] in (0, 1)
    if name == "c2c":
        r = oracle.check_one("counter", h)
        assert (r["valid"], r["explored"], r["fail_idx"]) == (gold["valid"], gold["explored"], gold["fail_idx"])


@pytest.mark.parametrize("name", ["ramp11s", "ramp10c17", "ramp11c17", "ramp13", "ramp14", "ramp16", "ramp13x50",
                                  "c4x15", "c4x15n", "c5xx2"])
def test_wide_fixtures_match_generator(name):
    """tests/golden/wide_<name>_oracle.json (tests/golden/pin_wide.py: real wide frontiers and
    full-size invalid runs) was made from this generator's history."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import pin_wide
    p = pin_wide.path_of(name)
    if not os.path.exists(p):
        pytest.skip(f"{name} not pinned")
    gold = json.load(open(p))
    h = pin_wide.GEN[name][2]()
    assert (h.n, h.n_ops()) == (gold["n_entries"], gold["n_ops"])
    assert pin_wide.digest(h) == gold["digest"]
    assert gold["err_code"] == 0 and gold["valid"] in (0, 1)
    if name.endswith(("x50", "x15n", "x2")):
        assert gold["valid"] == 0 and gold["fail_idx"] > 0  # a mid-history stop
    if name == "c4x15":  # (the perturbed read stayed explainable: a second full C4 count)
        assert gold["valid"] == 1 and gold["explored"] > 10 ** 10
