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
    assert L.lc_abi_version() == _lib.ABI_VERSION == 6


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


def test_synth_exact_crash_count():
    """The crash ramp's generator (tools/crash_ramp.py): exactly K write/cas ops crash, all in
    the first crash_span of the ops, the history stays linearizable, and n_crashed=None leaves
    the p_info draw (every BASELINE config's history) untouched."""
    for k in (0, 3, 9):
        h = synth.gen_register(400, 8, 0.01, 40 + k, n_crashed=k)
        info = np.nonzero(h.type == 3)[0]
        assert len(info) == k
        assert np.all(h.f[info] != 0)
        assert oracle.check_one("cas-register", h)["valid"] == 1
    a, b = synth.gen_register(300, 5, 0.05, 9), synth.gen_register(300, 5, 0.05, 9, n_crashed=None)
    for x, y in zip(a.arrays(), b.arrays()):
        assert np.array_equal(x, y)


def test_seeds_follow_survey():
    assert synth.seed_for(3, 7) == 0x5EED0000 + 3007


# ---- stored-history re-check (lincheck.edn / lincheck.recheck) ------

EDN_SAMPLE = r'''
{:type :invoke, :f :write, :value [0 3], :process 0, :time 10, :index 0}
#jepsen.history.Op{:index 1, :time 20, :type :ok, :process 0, :f :write, :value #jepsen.independent.Tuple{:key 0, :value 3}}
{:type :info, :f :start, :value nil, :process :nemesis, :index 2} ; a nemesis op
#_ {:ignored true}
{:type :invoke :f :cas :value [1 [3 4]] :process 1 :index 3 :error "x\"y" :x #{1 2} :y 1.5 :z \a}
'''


def _to_edn(x):
    from lincheck.history import KV
    if x is None:
        return "nil"
    if isinstance(x, KV):
        return f"[{_to_edn(x.key)} {_to_edn(x.value)}]"
    if isinstance(x, (list, tuple)):
        return "[" + " ".join(_to_edn(v) for v in x) + "]"
    if isinstance(x, str):
        return ":" + x
    return str(x)


def ops_to_edn(ops):
    return "\n".join("{" + ", ".join(f":{k} {_to_edn(v)}" for k, v in op.items()) + "}"
                     for op in ops) + "\n"


def test_edn_reader_sample():
    from lincheck import edn
    from lincheck.history import KV
    ops = edn.read_history(EDN_SAMPLE, independent=True)
    assert len(ops) == 4
    assert ops[0] == {"type": "invoke", "f": "write", "value": KV(0, 3), "process": 0,
                      "time": 10, "index": 0}
    assert ops[1]["value"] == KV(0, 3) and ops[1]["type"] == "ok"
    assert ops[2]["process"] == "nemesis" and ops[2]["value"] is None
    assert ops[3]["value"] == KV(1, [3, 4]) and ops[3]["error"] == 'x"y'
    assert ops[3]["x"] == frozenset({1, 2}) and ops[3]["y"] == 1.5 and ops[3]["z"] == "a"


def test_edn_vector_form_and_errors():
    from lincheck import edn
    ops = edn.read_history("[{:type :invoke :f :read :value nil :process 0}\n"
                           " {:type :ok :f :read :value 3 :process 0}]")
    assert [o["type"] for o in ops] == ["invoke", "ok"] and ops[1]["value"] == 3
    with pytest.raises(edn.EdnError):
        list(edn.loads_all("{:a 1"))


def test_edn_round_trip_independent_history(tmp_path):
    from lincheck import edn, history as H, synth
    from lincheck.history import KV
    h = synth.gen_register_keys(4, 60, 3, 0.05, config_id=1)
    ops = []
    for k in range(h.n_hist):
        for o in h.to_ops(k):
            o["value"] = KV(h.keys[k], o["value"])
            ops.append(o)
    ops.sort(key=lambda o: (o["index"], o["value"].key))
    p = tmp_path / "history.edn"
    p.write_text(ops_to_edn(ops))
    back = H.subhistories(edn.read_history(str(p), independent=True))
    want = H.subhistories(ops)
    assert back.keys == want.keys
    for a, b in zip(back.arrays(), want.arrays()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("n_shards", [1, 2, 3, 8])
def test_shard_histories_lpt(n_shards):
    """lc_shard_histories (the split lc_check(n_gpus > 1) and bench --gpus N use) runs without
    a device: every history lands on exactly one shard, deterministically, and the LPT bound
    holds: no shard exceeds the mean load by more than the largest history."""
    rng = np.random.default_rng(5)
    sizes = rng.integers(0, 400, 97)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    h = H.History(off, *(np.zeros(int(off[-1]), t) for t in
                         (np.int64, np.int32, np.int8, np.int8, np.int64, np.int64, np.int8)))
    a = _lib.shard_histories(h, n_shards)
    b = _lib.shard_histories(h, n_shards)
    assert np.array_equal(a, b)
    assert a.min() >= 0 and a.max() < n_shards
    load = np.bincount(a, weights=sizes, minlength=n_shards)
    assert load.max() <= sizes.sum() / n_shards + sizes.max()
    if n_shards == 1:
        assert np.all(a == 0)


def _live_widths_lff(h, k):
    """Per RETURN step, the live width of history k's table (lowest-free-first slots, crashed ops
    keep theirs): the encoder's slot policy never widens a table beyond it."""
    a, b = int(h.off[k]), int(h.off[k + 1])
    status, pend = {}, {}
    for i in range(a, b):
        p = int(h.process[i])
        if h.type[i] == 0:
            pend[p] = i
        else:
            status[pend.pop(p)] = int(h.type[i])
    used, slot, out = set(), {}, []
    pend = {}
    for i in range(a, b):
        p = int(h.process[i])
        if h.type[i] == 0:
            if status.get(i) == 2:  # failed ops never enter the search
                continue
            s = 0
            while s in used:
                s += 1
            used.add(s)
            slot[i] = s
            pend[p] = i
        elif h.type[i] == 1:
            inv = pend.pop(p)
            out.append(max(used) + 1)
            used.discard(slot[inv])
        elif p in pend:
            pend.pop(p)  # :info: the slot stays taken; :fail completions had no slot
    return out


@pytest.mark.parametrize("n_shards", [1, 2, 8])
def test_shard_histories_by_cost(n_shards):
    """lc_shard_histories_by_cost (lc_check(n_gpus > 1) and bench --gpus N): host only. The cost
    is each history's modeled chain time: for the C3 shape every key has ~2,000 entries, so the
    entry split is blind to it, while the modeled time follows the live widths (a step's table
    has 2^width masks). Every history on one shard, deterministic, LPT bound on the costs."""
    h = synth.gen_register_keys(64, 400, 5, 0.02, config_id=3)
    a, cost = _lib.shard_histories_by_cost(1, 0, h, n_shards)
    b, cost2 = _lib.shard_histories_by_cost(1, 0, h, n_shards)
    assert np.array_equal(a, b) and np.array_equal(cost, cost2)
    assert a.min() >= 0 and a.max() < n_shards and np.all(cost > 0)
    load = np.bincount(a, weights=cost, minlength=n_shards)
    assert load.max() <= cost.sum() / n_shards + cost.max() + 1e-6
    # the model per class (the team planner's fits): a WAVE history (width <= 11, one
    # wave: 7.9 us per step) costs more per step than a MID one (12..14, four waves: 4.9 us +
    # 0.0016 * 2^(L-3)), a BLOCK one (15..17) 4.67 + 0.00266 * 2^(L-3); widths as the encoder
    # gives them, no wider than lowest-free-first
    seen = set()
    for k in range(h.n_hist):
        ws = _live_widths_lff(h, k)
        n, lw = len(ws), max(ws)
        if lw <= 11:
            assert cost[k] == pytest.approx(7.9 * n), k
            seen.add("wave")
        elif lw <= 14:
            assert 4.9 * n <= cost[k] <= (4.9 + 0.0016 * 2 ** 11) * n, k
            seen.add("mid")
        elif lw <= 17:
            assert 4.67 * n <= cost[k] <= (4.67 + 0.00266 * 2 ** 14) * n, k
    assert seen == {"wave", "mid"}
    # counter histories balance by entry count
    c = H.concat([synth.gen_counter(n, 4, 0.0, 70 + n) for n in (50, 200, 100)])
    _, ccost = _lib.shard_histories_by_cost(2, 0, c, 2)
    assert list(ccost) == [float(c.off[k + 1] - c.off[k]) for k in range(3)]


def test_shard_cost_of_hbm_table_histories():
    """Histories of width 25..31 (the HBM tables) are priced per step as ~7 us of
    grid barriers plus their live words' bytes at 1.3 TB/s, not by entry count: the crash ramp's
    width-27/30 histories (K = 13, 16) cost tens to hundreds of ms, far above a C3 key, and LPT
    gives each its own shard."""
    hs = [synth.gen_register(2000, 16, 0.002, 0x5EED4000 + k, n_crashed=k) for k in (13, 16)]
    hs += [synth.gen_register(1000, 5, 0.01, 70 + k) for k in range(6)]
    h = H.concat(hs)
    shard, cost = _lib.shard_histories_by_cost(1, 0, h, 3)
    steps = [int(np.sum((h.sub(k).type == 1))) for k in range(2)]
    for k in range(2):
        assert cost[k] >= 7.0 * steps[k] * 0.5 and cost[k] > 5 * cost[2:].max(), (k, cost[k])
    assert 20_000 < cost[0] < 200_000 and 100_000 < cost[1] < 1_000_000  # us (measured 81 / 278 ms)
    assert shard[0] != shard[1] and not set(shard[2:]) & {shard[1]}


def test_shard_histories_rejects_bad_args():
    L = _lib.load()
    off = np.array([0, 5, 3], np.int64)  # not monotone
    out = np.zeros(2, np.int32)
    assert L.lc_shard_histories(2, _lib._p(off), 2, _lib._p(out)) == -1
    assert L.lc_shard_histories(2, _lib._p(np.array([0, 1, 2], np.int64)), 0, _lib._p(out)) == -1


def test_leader_model_is_searched_natively():
    """SURVEY §8(f) row 3, done natively since r3: LeaderModel (leader.clj:63-85) is model kind
    3 of the C ABI; only a Model(gpu=False) still gets the fallback map."""
    m = model.LeaderModel()
    assert m.gpu and m.kind == 3 and m.name == "leader"
    with pytest.raises(ValueError):
        model.LeaderModel({1: "n1"})
    r = checker.fallback_result(model.Model("other", 0, gpu=False))
    assert r["valid?"] == "unknown" and r["fallback"] == "knossos" and "error" in r


def test_leader_failure_report_shape_from_oracle_configs():
    """The checker's LeaderModel failure report, fed the oracle's pre-failure configs (the GPU
    test feeds the device's): configs carry term -> leader maps rebuilt from the returned and
    linearized ops, final paths end in the reference's message (leader.clj:73)."""
    import oracle
    from lincheck import synth
    done = 0
    for t in range(40):
        h = synth.gen_leader(60, 4, 0.1, 63000 + t, invalid=True, n_terms=3, p_crash=0.1)
        e = oracle.check_one("leader", h, with_configs=True)
        if e["valid"] != 0:
            continue
        r = {"valid": np.array([0]), "explored": np.array([e["explored"]]), "err": np.array([0]),
             "fail_idx": np.array([e["fail_idx"]]), "prev_ok": np.array([e["prev_ok_idx"]]),
             "fail_inv": np.array([e["fail_inv_idx"]])}
        cfgs = sorted(e["fail_configs"])
        lasts = [e["fail_last_op"][c] for c in cfgs]
        res = checker._result_map(h.to_ops(), r, 0, model.LeaderModel(),
                                  (cfgs, e["pending_inv_idx"], lasts, max(lasts)))
        op = res["op"]
        assert op["index"] == e["fail_idx"] and op["f"] == "inspect"
        for c in res["configs"]:
            m = c["model"]["value"]
            assert isinstance(m, dict) and all(isinstance(v, str) for v in m.values())
            # the failing op's term already has another leader in every config
            assert m.get(op["value"][1]) not in (None, op["value"][0])
        assert res["final-paths"]
        for p in res["final-paths"]:
            assert p[-1]["op"]["index"] == e["fail_inv_idx"]
            assert "but received" in p[-1]["model"]["inconsistent"]
        done += 1
    assert done > 5


def test_independent_failures_exclude_unknown():
    """jepsen.independent/checker lists keys whose :valid? is falsey; :unknown is truthy."""
    class Fixed(checker.Checker):
        def check(self, test, history, opts=None):
            return {"valid?": {0: True, 1: "unknown", 2: False}[history[0]["value"]]}
    ops = []
    for k in range(3):
        ops += [{"process": k, "type": "invoke", "f": "read", "value": H.KV(k, k), "index": 2 * k},
                {"process": k, "type": "ok", "f": "read", "value": H.KV(k, k), "index": 2 * k + 1}]
    r = checker.independent_checker(Fixed()).check({}, ops)
    assert r["failures"] == [2] and r["valid?"] is False


def _all_final_paths(model_name, cfgs, pending, fail_inv, ops, max_len):
    """Independent enumeration (brute.step): every sequence of pending ops from a config,
    each step consistent, ending with the failing op's inconsistent step (as op-index tuples)."""
    import brute
    folded = checker._folded_ops(ops)
    fop = folded[fail_inv]
    out = set()

    def val(s):
        return brute.NIL if s is None else s

    def go(cfg, state, lin, seq):
        if brute.step(model_name, state, fop["f"], fop["value"]) is None:
            out.add((cfg,) + tuple(seq))
        if len(seq) >= max_len:
            return
        for i in pending:
            if i in lin or i == fail_inv or i not in folded:
                continue
            o = folded[i]
            s2 = brute.step(model_name, state, o["f"], o["value"])
            if s2 is not None:
                go(cfg, s2, lin | {i}, seq + [i])
    for c, (s, lin) in enumerate(cfgs):
        go(c, val(s) if model_name == "cas-register" else s, frozenset(lin), [])
    return out


@pytest.mark.parametrize("model_name", ["cas-register", "counter"])
def test_final_paths_against_enumeration(model_name):
    """:final-paths: computed from the oracle's pre-failure configs, every
    path is one the independent enumeration finds (compared as sets), each ends with the failing
    op's inconsistent step, and the report holds min(10, all paths) of them, shortest first."""
    m = model.cas_register() if model_name == "cas-register" else model.CounterModel(0)
    gen = synth.gen_register if model_name == "cas-register" else synth.gen_counter
    seen = 0
    for t in range(40):
        h = gen(60, 4, 0.1, 9000 + t, invalid=True)
        e = oracle.check_one(model_name, h, with_configs=True)
        if e["valid"] != 0:
            continue
        ops = h.to_ops(0)
        cfgs = sorted(e["fail_configs"], key=lambda c: (c[0] is None, c[0] or 0, c[1]))[:10]
        paths = checker.final_paths(m, cfgs, e["pending_inv_idx"], e["fail_inv_idx"], ops)
        longest = max(len(p) for p in paths) - 2
        every = _all_final_paths(model_name, cfgs, e["pending_inv_idx"], e["fail_inv_idx"], ops, longest)
        got = set()
        for p in paths:  # (config, ops...) - the config recovered from the path's first model
            c = [i for i, (s_, lin) in enumerate(cfgs) if s_ == p[0]["model"]["value"]]
            got.add(next((i,) + tuple(x["op"]["index"] for x in p[1:-1]) for i in c
                         if (i,) + tuple(x["op"]["index"] for x in p[1:-1]) in every))
        assert got <= every
        assert len(paths) == min(10, len(_all_final_paths(model_name, cfgs, e["pending_inv_idx"],
                                                          e["fail_inv_idx"], ops, longest + 1)))
        for p in paths:
            assert p[0]["op"] is None and "inconsistent" in p[-1]["model"]
            assert p[-1]["op"]["index"] == e["fail_inv_idx"]
            assert all("value" in s_["model"] for s_ in p[:-1])
        # shortest first
        assert [len(p) for p in paths] == sorted(len(p) for p in paths)
        seen += 1
    assert seen >= 3
