"""GPU parity tests: the HIP search (through the C-ABI) against the CPU oracle on the same
seeded inputs, against the committed golden KATs, and — at BASELINE sizes — through
size-independent properties (determinism, perturbation detection, n_gpus invariance)."""
import json
import os
import random

import numpy as np
import pytest

import oracle
from brute import literal_search
from lincheck import _lib, checker, history as H, model, synth

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")))
KIND = {"cas-register": 1, "counter": 2, "leader": 3}


@pytest.fixture(scope="module", autouse=True)
def _device():
    if _lib.load().lc_device_count() < 1:
        pytest.fail("no HIP device on a GPU run: the checker has no CPU fallback")


def _cmp(got, exp, k=0, what=""):
    assert int(got["valid"][k]) == exp["valid"], (what, k, got["valid"][k], exp)
    assert int(got["fail_idx"][k]) == exp["fail_idx"], (what, k, got["fail_idx"][k], exp)
    assert int(got["fail_inv"][k]) == exp["fail_inv_idx"], (what, k)
    assert int(got["prev_ok"][k]) == exp["prev_ok_idx"], (what, k)
    if exp["valid"] != 2:
        assert int(got["explored"][k]) == exp["explored"], (what, k, got["explored"][k], exp)


@pytest.mark.parametrize("kat", GOLD, ids=[k["name"] for k in GOLD])
def test_gpu_kats(kat):
    h = H.encode(kat["history"])
    g = _lib.check(KIND[kat["model"]], 0, h)
    assert int(g["valid"][0]) == (1 if kat["valid"] else 0)
    assert int(g["fail_idx"][0]) == kat["fail_idx"]
    if kat["prev_ok_idx"] is not None:
        assert int(g["prev_ok"][0]) == kat["prev_ok_idx"]
    if kat["explored"] is not None:
        assert int(g["explored"][0]) == kat["explored"]


def test_gpu_kats_batched():
    """All KATs of one model in one call: batching must not change any answer."""
    for m in ("cas-register", "counter"):
        kats = [k for k in GOLD if k["model"] == m]
        h = H.concat([H.encode(k["history"]) for k in kats])
        g = _lib.check(KIND[m], 0, h)
        for i, k in enumerate(kats):
            assert int(g["valid"][i]) == (1 if k["valid"] else 0), k["name"]
            assert int(g["fail_idx"][i]) == k["fail_idx"], k["name"]


@pytest.mark.parametrize("m", ["cas-register", "counter"])
def test_gpu_random_small_vs_oracle(m):
    rng = random.Random(11)
    gen = synth.gen_register if m == "cas-register" else synth.gen_counter
    hs = [gen(rng.randint(1, 40), rng.randint(1, 6), 0.2, 4000 + t, invalid=(t % 2 == 1))
          for t in range(300)]
    h = H.concat(hs)
    g = _lib.check(KIND[m], 0, h)
    exp = oracle.check_many(m, h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, m)
    assert any(e["valid"] == 0 for e in exp) and any(e["valid"] == 1 for e in exp)


def test_gpu_c1_vs_oracle():
    """BASELINE config C1: 10 keys x 200 ops, 5 clients."""
    h = synth.gen_config("c1")
    g = _lib.check(1, 0, h)
    exp = oracle.check_many("cas-register", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, "c1")


def test_gpu_c3_subset_vs_oracle():
    """C3 shape (1k ops/key, 5 clients, p_info 0.01) on 24 keys, 4 perturbed."""
    h = synth.gen_register_keys(24, 1000, 5, 0.01, config_id=3, invalid_keys=(2, 5, 11, 17))
    g = _lib.check(1, 0, h)
    exp = oracle.check_many("cas-register", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, "c3-subset")


def test_gpu_c2_scaled_vs_oracle():
    """C2 shape (1 key, 16 clients, p_info 0.002): deep frontier, spills the LDS tables."""
    h = synth.gen_register(1500, 16, 0.002, synth.seed_for(2, 0))
    g = _lib.check(1, 0, h)
    _cmp(g, oracle.check_one("cas-register", h), 0, "c2-scaled")


def test_gpu_c2_full_size_vs_oracle():
    """BASELINE config C2 at full size (1 key x 5k ops, 16 clients): every one of its 10,000
    entries, bit-exact with the oracle (verdict, indices, explored)."""
    h = synth.gen_config("c2")
    assert h.n == int(h.off[-1]) and h.n_ops() == 5000
    g = _lib.check(1, 0, h)
    _cmp(g, oracle.check_one("cas-register", h), 0, "c2-full")


# C4 (BASELINE configs[3]): one 100k-op history with crashed :info ops. Its full-size oracle
# verdict and explored count (tests/golden/c4_oracle.json: the C oracle on one thread, 3.0 h,
# made by tests/golden/pin_c4.py) are the fixture every GPU path must reproduce.
C4_GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "c4_oracle.json")))
C4_EXPLORED = C4_GOLD["explored"]
assert C4_GOLD["valid"] == 1 and C4_GOLD["err_code"] == 0 and C4_GOLD["n_ops"] == 100_000


def test_gpu_c4_full_size_grid(monkeypatch):
    monkeypatch.setenv("LC_PATH", "grid")
    h = synth.gen_config("c4")
    assert h.n_ops() == 100_000
    g = _lib.check(1, 0, h)
    assert int(g["err"][0]) == 0 and int(g["valid"][0]) == 1
    assert int(g["explored"][0]) == C4_EXPLORED


def test_gpu_lc_check_env_knobs_do_not_stick(monkeypatch):
    """lc_check reuses one cached plan per device; a knob set for one call
    (LC_PATH=grid, capacity test hooks) must not carry into the next call without it."""
    h = synth.gen_register_keys(6, 200, 5, 0.01, config_id=3)
    monkeypatch.setenv("LC_PATH", "grid")
    monkeypatch.setenv("LC_CELLCAP", "4")
    g1 = _lib.check(1, 0, h)
    assert _lib.check_stats(0)["dense_histories"] == 0
    monkeypatch.delenv("LC_PATH")
    monkeypatch.delenv("LC_CELLCAP")
    g2 = _lib.check(1, 0, h)
    assert _lib.check_stats(0)["dense_histories"] == h.n_hist
    for k in g1:
        assert np.array_equal(g1[k], g2[k]), k
    _lib.release(0)  # lc_release: the next call rebuilds the cached plan
    g3 = _lib.check(1, 0, h)
    assert _lib.check_stats(0)["dense_histories"] == h.n_hist
    for k in g1:
        assert np.array_equal(g1[k], g3[k]), k


def test_gpu_c4_full_size_dense():
    """C4 on the dense closure tables (the default path since steps carry 24 live slots): a
    pipelined tile team of up to 2^7 workgroups; the same explored count as the grid kernel."""
    h = synth.gen_config("c4")
    p = _lib.Plan(1, 0, h)
    p.run()
    g = p.results()
    s = p.stats()
    p.close()
    assert s["dense_histories"] == 1
    assert int(g["err"][0]) == 0 and int(g["valid"][0]) == 1
    assert int(g["explored"][0]) == C4_EXPLORED


@pytest.mark.parametrize("flow", ["1", "0"], ids=["flow", "levels"])
def test_gpu_c4_full_size_partitioned_world1(flow, monkeypatch):
    from lincheck import partition
    monkeypatch.setenv("LC_PART_FLOW", flow)
    h = synth.gen_config("c4")
    r = partition.check_partitioned(h, capacity_log2=25)
    assert (r["valid"], r["err"], r["explored"]) == (1, 0, C4_EXPLORED)


def test_gpu_c4_prefix_vs_oracle():
    """The C4 history's first 16k entries and a perturbed C4-shaped history vs the oracle."""
    h = synth.gen_config("c4")
    p = synth.truncate(h, 16_000)  # ~11 s of oracle time
    g = _lib.check(1, 0, p)
    _cmp(g, oracle.check_one("cas-register", p), 0, "c4-prefix")
    # the same prefix with a tail no linearization explains (a fresh client writes 9, reads 9,
    # then reads 7, a value no op writes): caught at that :ok, with the prefix's explored count
    n0 = p.n
    tail = [(9001, 0, 1, 1, 9), (9001, 1, 1, 1, 9), (9002, 0, 0, 0, 0), (9002, 1, 0, 1, 9),
            (9003, 0, 0, 0, 0), (9003, 1, 0, 1, 7)]  # (process, type, f, vflags, v0)
    cols = [np.concatenate([a, np.array(b, a.dtype)]) for a, b in zip(
        (p.index, p.process, p.type, p.f, p.v0, p.v1, p.vflags),
        (np.arange(n0, n0 + len(tail)), [t[0] for t in tail], [t[1] for t in tail],
         [t[2] for t in tail], [t[4] for t in tail], [0] * len(tail), [t[3] for t in tail]))]
    bad = H.from_columns(*cols)
    gb = _lib.check(1, 0, bad)
    eb = oracle.check_one("cas-register", bad)
    assert eb["valid"] == 0 and eb["fail_idx"] == n0 + 5
    _cmp(gb, eb, 0, "c4-prefix-invalid-tail")


def test_gpu_lc_check_shards_multiplexed():
    """lc_check(n_gpus > 1): the LPT split, one thread per shard and the scatter of results
    back to history order. More shards than devices run multiplexed on the visible ones, so a
    1-GPU box exercises the whole multi-device path; answers do not depend on n_gpus."""
    h = synth.gen_register_keys(40, 400, 5, 0.02, config_id=3, invalid_keys=(3, 17, 29))
    ref = _lib.check(1, 0, h, n_gpus=1)
    for n in (2, 3, 8):
        g = _lib.check(1, 0, h, n_gpus=n)
        for k in ref:
            assert np.array_equal(ref[k], g[k]), (n, k)
    exp = oracle.check_many("cas-register", h)
    for k in range(h.n_hist):
        _cmp(ref, exp[k], k, "sharded")


def test_gpu_counter_vs_oracle():
    hs = [synth.gen_counter(400, 6, 0.005, 9000 + t, invalid=(t % 3 == 0)) for t in range(12)]
    h = H.concat(hs)
    g = _lib.check(2, 0, h)
    exp = oracle.check_many("counter", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, "counter")


def test_gpu_counter_init_value():
    h = synth.gen_counter(200, 4, 0.0, 5)
    for init in (0, 7, -3):
        g = _lib.check(2, init, h)
        _cmp(g, oracle.check_one("counter", h, init_value=init), 0, f"init={init}")


@pytest.mark.parametrize("m", ["cas-register", "counter"])
def test_gpu_failure_configs_match_oracle(m):
    found = carried = 0
    gen = synth.gen_register if m == "cas-register" else synth.gen_counter
    for t in range(30):
        h = gen(80, 4, 0.1, 9000 + t, invalid=True)
        g = _lib.check(KIND[m], 0, h)
        e = oracle.check_one(m, h, with_configs=True)
        assert int(g["valid"][0]) == e["valid"]
        if e["valid"] != 0:
            continue
        cfgs, pending, lasts, newest = _lib.failure_configs(0, 1 << 12, with_last=True)
        assert sorted(pending) == sorted(e["pending_inv_idx"])
        assert set(cfgs) == e["fail_configs"]
        assert len(cfgs) == len(e["fail_configs"])
        # per-config :last-op (Knossos's :configs entries) from the search's tags
        for c, last in zip(cfgs, lasts):
            assert last == e["fail_last_op"][c], (t, c, last, e["fail_last_op"][c])
        assert newest == max(e["fail_last_op"].values())
        carried += sum(1 for x in lasts if x != e["prev_ok_idx"])
        found += 1
    assert found > 5 and carried > 0  # some configs were carried through the last RETURN


def test_gpu_failure_configs_untagged_fallback():
    """a key with no room for the 6-bit last-op tag (here 56 calls pending + 3 state
    bits) still gets its :configs, untagged: the same configs as the oracle's, each with the
    previous :ok op as its :last-op (the report's no-tag rendering)."""
    for t in range(8):
        base = synth.gen_register(40, 3, 0.0, 9100 + t, invalid=True)
        h = _with_never_ops(base, 52)
        g = _lib.check(1, 0, h)
        e = oracle.check_one("cas-register", h, with_configs=True)
        assert int(g["valid"][0]) == e["valid"]
        if e["valid"] != 0:
            continue
        cfgs, pending, lasts, newest = _lib.failure_configs(0, 1 << 12, with_last=True)
        assert set(cfgs) == e["fail_configs"] and len(cfgs) == len(e["fail_configs"])
        assert sorted(pending) == sorted(e["pending_inv_idx"])
        assert all(x == e["prev_ok_idx"] for x in lasts) and newest == e["prev_ok_idx"]
        return
    pytest.fail("no invalid history among the seeds")


def _leader_hists(n, seed0, n_ops=200, p_crash=0.03):
    return [synth.gen_leader(n_ops, 5, 0.05, seed0 + t, invalid=(t % 3 == 1), n_terms=4 + t % 5,
                             p_crash=p_crash if t % 2 else 0.0) for t in range(n)]


@pytest.mark.parametrize("path", [None, "keys", "grid"])
def test_gpu_leader_vs_oracle(path, monkeypatch):
    """The :election workload's LeaderModel (leader.clj:63-85) on the GPU search: verdicts,
    failing ops and explored counts bit-exact with the oracle, invalid histories (a second
    leader in one term) and crashed ops (pending forever with [nil 0]) included, through the
    per-key kernel and the grid kernel."""
    if path:
        monkeypatch.setenv("LC_PATH", path)
    h = H.concat(_leader_hists(30, 62000))
    g = _lib.check(3, 0, h)
    exp = oracle.check_many("leader", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"leader path={path}")
    assert any(e["valid"] == 0 for e in exp) and any(e["valid"] == 1 for e in exp)


def test_gpu_leader_contested_pair_limit():
    """More than 64 contested (term, leader) pairs: :unknown with the capacity code (the
    oracle, whose limit counts every distinct pair, cannot check such a history either)."""
    ops = []
    for t in range(33):  # 33 terms, two leaders each: 66 contested pairs
        for p, name in ((0, "a"), (1, "b")):
            ops += [{"process": p, "type": "invoke", "f": "inspect", "value": [None, 0]},
                    {"process": p, "type": "ok", "f": "inspect", "value": [name, t + 1]}]
    g = _lib.check(3, 0, H.encode(ops))
    assert int(g["valid"][0]) == 2 and int(g["err"][0]) == -7


def test_gpu_leader_failure_report():
    """Failure report for LeaderModel: the pre-failure configs (as linearized sets: the
    device holds contested pairs, the oracle every pair) and per-config :last-op match the
    oracle; the checker's map carries term -> leader maps and final paths ending in the
    reference's inconsistency message."""
    from lincheck import checker, model
    found = 0
    for t in range(30):
        h = synth.gen_leader(60, 4, 0.1, 63000 + t, invalid=True, n_terms=3, p_crash=0.1)
        e = oracle.check_one("leader", h, with_configs=True)
        g = _lib.check(3, 0, h)
        assert int(g["valid"][0]) == e["valid"]
        if e["valid"] != 0:
            continue
        cfgs, pending, lasts, newest = _lib.failure_configs(0, 1 << 12, with_last=True)
        assert sorted(pending) == sorted(e["pending_inv_idx"])
        got = {lin: last for (_s, lin), last in zip(cfgs, lasts)}
        want = {lin: e["fail_last_op"][(s, lin)] for (s, lin) in e["fail_configs"]}
        assert got == want and len(cfgs) == len(e["fail_configs"])
        res = checker.linearizable({"model": model.LeaderModel()}).check({}, h.to_ops(), {})
        assert res["valid?"] is False and res["op"]["index"] == e["fail_idx"]
        for c in res["configs"]:
            assert isinstance(c["model"]["value"], dict)
        assert res["final-paths"] and all("but received" in p[-1]["model"]["inconsistent"]
                                          for p in res["final-paths"])
        found += 1
    assert found > 5


def test_gpu_counter_bounds_vs_oracle():
    for t in range(40):
        h = synth.gen_counter(300, 5, 0.05, 600 + t, invalid=(t % 2 == 0))
        ok, bad = _lib.counter_bounds(0, h)
        eok, ebad = oracle.counter_bounds(h)
        assert bool(ok[0]) == eok and int(bad[0]) == ebad


def test_gpu_counter_bounds_c5_full_size():
    """C5 size (1M ops): the scan must accept the linearizable history and reject a
    perturbed read (size-independent property: soundness + detection)."""
    h = synth.gen_config("c5")
    ok, bad = _lib.counter_bounds(0, h)
    eok, ebad = oracle.counter_bounds(h)
    assert bool(ok[0]) and eok
    # perturb one read far outside any window
    reads = np.nonzero((h.type == 1) & (h.f == 0))[0]
    j = reads[len(reads) // 2]
    h.v0[j] += 10 ** 6
    ok, bad = _lib.counter_bounds(0, h)
    eok, ebad = oracle.counter_bounds(h)
    assert not ok[0] and not eok and int(bad[0]) == ebad


def _sharded_bounds(h, world):
    """Scan one counter history as `world` shards on one GPU: every shard's block sums, the
    exclusive prefix an all-gather would give each, then each shard's run (lincheck.shard)."""
    from lincheck import shard
    n = int(h.off[1] - h.off[0])
    plans = [_lib.BoundsPlan(0, h, own=shard.bounds_shard(n, r, world)) for r in range(world)]
    sums = [p.sums() for p in plans]
    bad = -1
    try:
        for r, p in enumerate(plans):
            excl = np.sum(sums[:r], axis=0) if r else np.zeros(5, np.int64)
            ok, b, ms = p.run(excl)
            assert ok == (b < 0) and ms >= 0
            if b >= 0 and (bad < 0 or b < bad):
                bad = b
    finally:
        for p in plans:
            p.close()
    return bad < 0, bad


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_gpu_bounds_plan_shards_vs_oracle(world):
    for t in range(24):
        h = synth.gen_counter(400, 5, 0.05, 900 + t, invalid=(t % 2 == 0))
        ok, bad = _sharded_bounds(h, world)
        eok, ebad = oracle.counter_bounds(h)
        assert ok == eok and bad == ebad, (world, t)


def test_gpu_bounds_plan_c5_full_size_sharded():
    h = synth.gen_config("c5")
    reads = np.nonzero((h.type == 1) & (h.f == 0))[0]
    for world in (1, 8):
        assert _sharded_bounds(h, world) == (True, -1)
    j = reads[(3 * len(reads)) // 4]
    h.v0[j] += 10 ** 6
    eok, ebad = oracle.counter_bounds(h)
    assert not eok
    for world in (1, 8):
        assert _sharded_bounds(h, world) == (False, ebad)


def test_gpu_bounds_plan_empty_and_tiny():
    for ev in ([], [{"process": 0, "type": "invoke", "f": "read", "value": None},
                    {"process": 0, "type": "ok", "f": "read", "value": 3}]):
        h = H.encode(ev)
        eok, ebad = oracle.counter_bounds(h)
        assert _sharded_bounds(h, 1) == (eok, ebad)


def test_gpu_errors_are_unknown():
    bad = H.encode([{"process": 0, "type": "ok", "f": "read", "value": 1}])
    g = _lib.check(1, 0, bad)
    assert int(g["valid"][0]) == 2 and int(g["err"][0]) == -4
    wrong_f = H.encode([{"process": 0, "type": "invoke", "f": "cas", "value": [1, 2]},
                        {"process": 0, "type": "ok", "f": "cas", "value": [1, 2]}])
    g = _lib.check(2, 0, wrong_f)
    assert int(g["valid"][0]) == 2 and int(g["err"][0]) == -6
    ovf = H.encode([{"process": 0, "type": "invoke", "f": "add", "value": 2 ** 62},
                    {"process": 0, "type": "ok", "f": "add", "value": 2 ** 62},
                    {"process": 1, "type": "invoke", "f": "add", "value": 2 ** 62},
                    {"process": 1, "type": "ok", "f": "add", "value": 2 ** 62}])
    g = _lib.check(2, 0, ovf)
    e = oracle.check_one("counter", ovf)
    assert e["valid"] == 2 and int(g["valid"][0]) == 2 and int(g["err"][0]) == -6


def test_gpu_deterministic_and_plan_reuse():
    h = synth.gen_register_keys(64, 500, 5, 0.01, config_id=7, invalid_keys=(9,))
    p = _lib.Plan(1, 0, h)
    p.run()
    r1 = p.results()
    p.run()
    r2 = p.results()
    for k in r1:
        assert np.array_equal(r1[k], r2[k]), k
    r3 = _lib.check(1, 0, h)
    for k in r1:
        assert np.array_equal(r1[k], r3[k]), k
    s = p.stats()
    assert s["kernel_ms"] > 0 and s["alg_bytes"] > 0 and s["closure_new"] == r1["explored"].sum()
    p.close()


def test_gpu_c3_full_size_vs_oracle():
    """C3 at full size (1k keys x 1k ops, BASELINE configs[2]), three keys perturbed: all 1000
    keys bit-exact with the oracle (verdict, failing :ok, its invocation, :previous-ok,
    explored; ~20 s of oracle time on 16 threads), and n_gpus does not change answers."""
    h = synth.gen_register_keys(1000, 1000, 5, 0.01, config_id=3, invalid_keys=(1, 500, 999))
    g = _lib.check(1, 0, h)
    assert np.all(g["err"] == 0)
    exp = oracle.check_many("cas-register", h, n_threads=16)
    for k in range(1000):
        _cmp(g, exp[k], k, "c3-full")
    clean = np.ones(1000, bool)
    clean[[1, 500, 999]] = False
    assert np.all(g["valid"][clean] == 1)
    g2 = _lib.check(1, 0, h, n_gpus=0)
    for k in g:
        assert np.array_equal(g[k], g2[k])


def test_checker_api_register_independent():
    ops = []
    idx = 0
    for key in range(3):
        for (p, t, f, v) in [(0, "invoke", "write", 1), (0, "ok", "write", 1),
                             (1, "invoke", "read", None), (1, "ok", "read", 1 if key != 1 else 2)]:
            ops.append({"process": p + 10 * key, "type": t, "f": f, "value": H.tuple_(key, v),
                        "index": idx})
            idx += 1
    c = checker.independent_checker(checker.compose({
        "timeline": checker.timeline_html(),
        "linear": checker.linearizable({"model": model.cas_register(), "algorithm": "linear"})}))
    r = c.check({}, ops, {})
    assert r["valid?"] is False and r["failures"] == [1]
    assert r["results"][0]["valid?"] is True
    lin = r["results"][1]["linear"]
    assert lin["valid?"] is False and lin["op"]["index"] == 7 and lin["previous-ok"]["index"] == 5
    assert lin["configs"] and all(cfg["model"]["value"] == 1 for cfg in lin["configs"])
    # Knossos-shaped :configs [ext]: {:model :last-op :pending}; the write (index 5) is the only
    # linearized op, so every config has it last and nothing pending but the failing read
    for cfg in lin["configs"]:
        assert set(cfg) == {"model", "last-op", "pending"}
        assert cfg["last-op"]["index"] == 5 and cfg["last-op"]["type"] == "ok"
        assert [o["index"] for o in cfg["pending"]] == [6]
    assert lin["last-op"]["index"] == 5


def test_checker_api_counter_kats():
    for kat in [k for k in GOLD if k["model"] == "counter" and k["name"].startswith("counter_")]:
        c = checker.linearizable({"model": model.CounterModel(0), "algorithm": "linear"})
        r = c.check({}, kat["history"], {})
        assert r["valid?"] is kat["valid"], kat["name"]


def _live_width(h, k):
    """Widest live-slot window (lowest-free-first slots, crashed ops keep theirs) of history k:
    the table width the dense kernel needs."""
    a, b = int(h.off[k]), int(h.off[k + 1])
    comp, pend = {}, {}
    for i in range(a, b):
        p = int(h.process[i])
        if h.type[i] == 0:
            pend[p] = i
        else:
            comp[pend.pop(p)] = int(h.type[i])
    used, slot, width = set(), {}, 0
    for i in range(a, b):
        p = int(h.process[i])
        if h.type[i] == 0:
            if comp.get(i) == 2:
                continue
            s = 0
            while s in used:
                s += 1
            used.add(s)
            slot[p] = s
            width = max(width, max(used) + 1)
        elif h.type[i] == 1:
            used.discard(slot.pop(p))
        elif h.type[i] == 3:
            slot.pop(p, None)
    return width


def test_gpu_dense_tables_vs_oracle():
    """Dense closure tables (dense.hip): wave teams (width <= 11), workgroup teams (12..17)
    and wide teams (18..22, HBM tables), in one batch, bit-exact with the oracle."""
    hs = [synth.gen_register_keys(28, 1000, 5, 0.01, config_id=3, invalid_keys=(2, 9, 20))]
    hs += [synth.gen_register(150, 5, 0.12, 31000 + t, invalid=(t % 2 == 0)) for t in range(6)]
    h = H.concat(hs)
    widths = [_live_width(h, k) for k in range(h.n_hist)]
    assert min(widths) <= 12 and any(13 <= w <= 17 for w in widths) and max(widths) > 17
    p = _lib.Plan(1, 0, h)
    p.run()
    g = p.results()
    s = p.stats()
    assert s["dense_histories"] == sum(w <= 22 for w in widths)
    exp = oracle.check_many("cas-register", h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"dense w={widths[k]}")
    assert any(e["valid"] == 0 for e in exp)
    p.close()


@pytest.mark.parametrize("plan", ["1", "0"])
def test_gpu_dense_team_planner(plan, monkeypatch):
    """The team planner (LC_PIPE bits 2|3, the default): with few histories per GPU (as each
    rank holds when C3's keys are split over 8 GPUs) the longest ones get smaller tiles, and
    BLOCK-width histories (15..17) become 2-tile teams. Bit-exact with the oracle and with the
    planner off (LC_TEAM_PLAN=0: 17-bit tiles for width > 17 only)."""
    monkeypatch.setenv("LC_TEAM_PLAN", plan)
    h = H.concat([synth.gen_register_keys(14, 1000, 5, 0.01, config_id=3, key0=250)] +
                 [synth.gen_register(150, 5, 0.12, 31000 + t, invalid=True) for t in (0, 2, 5, 6)])
    widths = [_live_width(h, k) for k in range(h.n_hist)]
    assert any(15 <= w <= 17 for w in widths) and max(widths) > 17
    g = _lib.check(1, 0, h)
    exp = oracle.check_many("cas-register", h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"plan={plan} w={widths[k]}")
    assert any(e["valid"] == 0 for e in exp)


@pytest.mark.parametrize("pipe", ["0", "1", "2", "3", "11", "15", "27", "47", "79", "143", "207",
                                  "515", "539", "591", "719", "975", "1999", "3139", "4047", "8143",
                                  "12239", "20431", "28623", "85967", "217039"])
def test_gpu_dense_pipelined_steps(pipe, monkeypatch):
    """LC_PIPE bit 0 / bit 1: BLOCK / WAVE teams overlap consecutive RETURN steps (step t+1's
    layer q beside step t's layer q + 2, returns read through the previous step's slot, fresh
    slots masked). Every mode is bit-exact with the oracle, invalid histories included (the
    failing step is found from the next step's empty frontier). 11 adds barrier-free tile teams
    (the default), 27 also MID teams (widths 12..14 on 256-thread workgroups); 79 WAVE
    histories on the big kernel's waves, 143/207 MID histories as 4-wave teams inside big
    workgroups (LDS barriers of their own). +512: double-buffered tables (a step after an
    in-word return starts one super-layer after its predecessor). +1024: WAVE histories of at most
    9 slots in one wave's registers (lane shuffles); +2048: their closure as a whole-table
    fixpoint instead of the popcount-layer DP."""
    monkeypatch.setenv("LC_PIPE", pipe)
    hs = [synth.gen_register_keys(24, 600, 5, 0.01, config_id=3, invalid_keys=(1, 7, 16))]
    hs += [synth.gen_register(120, 5, 0.1, 33000 + t, invalid=(t % 2 == 1)) for t in range(8)]
    hs += [synth.gen_register(40, 3, 0.0, 34000 + t, invalid=(t % 3 == 0)) for t in range(6)]
    h = H.concat(hs)
    widths = [_live_width(h, k) for k in range(h.n_hist)]
    assert min(widths) <= 11 and any(12 <= w <= 17 for w in widths)
    p = _lib.Plan(1, 0, h)
    p.run()
    g = p.results()
    exp = oracle.check_many("cas-register", h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"pipe={pipe} w={widths[k]}")
    assert any(e["valid"] == 0 for e in exp)
    p.close()


def _low_slot_rounds(n_rounds, seed, perturb=False):
    """Rounds of four overlapping calls: slots 0..2 and 3 invoked together, slot 3 returns
    first (a hi-bit RETURN with all three low ops live), then 0..2 in a random order. Writes,
    cas and reads over values 0..2 take effect in a random permutation of the round, so the
    in-word closure must reach every ordering of the three low ops (writes are OR-folds)."""
    rng = random.Random(seed)
    ops, val = [], None
    for _ in range(n_rounds):
        calls = []
        for p in range(4):
            f = rng.choice(["write", "cas", "read", "write"])
            calls.append([p, f, rng.randrange(3) if f == "write" else [rng.randrange(3), rng.randrange(3)] if f == "cas" else None])
        for p, f, v in calls:
            ops.append({"process": p, "type": "invoke", "f": f, "value": v})
        done = {}
        for i in rng.sample(range(4), 4):  # the linearization order of this round
            p, f, v = calls[i]
            if f == "write":
                val, done[p] = v, ("ok", v)
            elif f == "read":
                done[p] = ("ok", val)
            else:
                ok = val == v[0]
                if ok:
                    val = v[1]
                done[p] = ("ok" if ok else "fail", v)
        for p in [3] + rng.sample(range(3), 3):
            t, v = done[p]
            if perturb and calls[p][1] == "read" and t == "ok" and rng.random() < 0.3:
                v = ((v if v is not None else -1) + 1) % 3
            ops.append({"process": p, "type": t, "f": calls[p][1], "value": v})
    return H.encode(ops)


@pytest.mark.parametrize("pipe", ["0", "11", "207", "719", "975", "1999", "4047", "8143"])
def test_gpu_dense_low_slot_orderings(pipe, monkeypatch):
    """The in-word closure's op sequence (0 1 2 0 1 0 2 for three live low ops, a b a for two):
    RETURNs of slot 3 with slots 0..2 pending, writes among them; bit-exact with the oracle,
    perturbed variants included, through the WAVE teams' per-step and pipelined loops."""
    monkeypatch.setenv("LC_PIPE", pipe)
    h = H.concat([_low_slot_rounds(60, 71000 + t, perturb=(t % 2 == 1)) for t in range(16)])
    exp = oracle.check_many("cas-register", h, n_threads=8)
    assert any(e["valid"] == 0 for e in exp) and any(e["valid"] == 1 for e in exp)
    g = _lib.check(1, 0, h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, "low-slot orderings")


_WIDE = {}


def _wide_batch():
    """Short histories with many crashed ops: live widths 18..22 (wide teams), with their
    oracle results (computed once per module)."""
    if _WIDE:
        return _WIDE["h"], _WIDE["widths"], _WIDE["exp"]
    hs, widths = [], []
    for t in range(60):
        h = synth.gen_register(130, 5, 0.15, 52000 + t, invalid=(t % 3 == 0))
        w = _live_width(h, 0)
        if 18 <= w <= 22:
            hs.append(h)
            widths.append(w)
        if len(hs) == 6:
            break
    assert len(hs) >= 4, widths
    h = H.concat(hs)
    _WIDE.update(h=h, widths=widths, exp=oracle.check_many("cas-register", h, n_threads=8))
    return h, widths, _WIDE["exp"]


@pytest.mark.parametrize("cap", [None, "8", "1"])
def test_gpu_dense_tile_teams(cap, monkeypatch):
    """Tile teams (width 18..22): 2^(width-17) workgroups, one 17-bit LDS tile each; cross-tile
    pulls through HBM mirrors and per-layer tokens, team-slot returns through the mirrors.
    Packing the teams into several launches (LC_TILE_WGS) must not change answers."""
    if cap:
        monkeypatch.setenv("LC_TILE_WGS", cap)
    h, widths, exp = _wide_batch()
    p = _lib.Plan(1, 0, h)
    p.run()
    got = p.results()
    s = p.stats()
    assert s["dense_histories"] == h.n_hist
    if cap == "1":
        assert s["launches"] >= h.n_hist  # one launch per team
    for k in range(h.n_hist):
        _cmp(got, exp[k], k, f"tile cap={cap} w={widths[k]}")
    p.close()


def test_gpu_dense_tile_teams_with_step_barriers(monkeypatch):
    """LC_PIPE=3: the tile-team loop with a leader command and a team barrier per team step
    (the default, bit 3, drops both and decides survivors from per-step bits after the last
    step): same answers."""
    monkeypatch.setenv("LC_PIPE", "3")
    h, widths, exp = _wide_batch()
    p = _lib.Plan(1, 0, h)
    p.run()
    got = p.results()
    for k in range(h.n_hist):
        _cmp(got, exp[k], k, f"barrier team loop w={widths[k]}")
    p.close()


@pytest.mark.parametrize("lbits", ["16", "15", "14", "12"])
def test_gpu_dense_tile_teams_small_tiles(lbits, monkeypatch):
    """The default (barrier-free) tile-team loop with smaller tiles: up to 2^8 workgroups per
    team, so the "every tile finished step s - 2" check spans several 64-lane chunks."""
    monkeypatch.setenv("LC_TILE_LBITS", lbits)
    h, widths, exp = _wide_batch()
    p = _lib.Plan(1, 0, h)
    p.run()
    got = p.results()
    for k in range(h.n_hist):
        _cmp(got, exp[k], k, f"small tiles lbits={lbits} w={widths[k]}")
    p.close()


@pytest.mark.parametrize("pipe", ["207", "463", "719", "975"],
                         ids=["tokens", "tagged", "tokens-dbl", "tagged-dbl"])
@pytest.mark.parametrize("rot,lbits", [("1", "14"), ("3", "13"), ("9", "15"), ("9", None)])
def test_gpu_dense_tile_teams_rotated(rot, lbits, pipe, monkeypatch):
    """LC_TEAM_ROT: a tile team's lowest slots relabelled as its team bits (every tile holds a
    share of every step). Slot labels are arbitrary, so every answer stays the oracle's. With
    LC_PIPE 463 the team mirrors are tagged words polled by their readers (no tokens)."""
    monkeypatch.setenv("LC_TEAM_ROT", rot)
    monkeypatch.setenv("LC_PIPE", pipe)
    if lbits:
        monkeypatch.setenv("LC_TILE_LBITS", lbits)
    h, widths, exp = _wide_batch()
    p = _lib.Plan(1, 0, h)
    p.run()
    got = p.results()
    for k in range(h.n_hist):
        _cmp(got, exp[k], k, f"rotated {rot} lbits={lbits} w={widths[k]}")
    p.close()


@pytest.mark.parametrize("pipe", ["11983", "12239"], ids=["tokens", "tagged"])
@pytest.mark.parametrize("rot,lbits", [("0", None), ("0", "15"), ("0", "14"), ("9", None), ("9", "14"), ("2", "15")])
def test_gpu_dense_tile_teams_global_layers(rot, lbits, pipe, monkeypatch):
    """LC_PIPE bit 13: a wide step's tile r runs its local layer q at super-layer
    start + q + |r| (global popcount layers), so cross-tile pulls read the previous super-layer
    and a step spans H + T + 1 super-layers. Same answers, unrotated and rotated, with tokens
    (11983) or tagged mirror words (12239), on teams of 2 to 256 tiles."""
    monkeypatch.setenv("LC_TEAM_ROT", rot)
    monkeypatch.setenv("LC_PIPE", pipe)
    if lbits:
        monkeypatch.setenv("LC_TILE_LBITS", lbits)
    h, widths, exp = _wide_batch()
    p = _lib.Plan(1, 0, h)
    p.run()
    got = p.results()
    for k in range(h.n_hist):
        _cmp(got, exp[k], k, f"global layers rot={rot} lbits={lbits} w={widths[k]}")
    p.close()


@pytest.mark.parametrize("lbits", [None, "15"])
def test_gpu_dense_tile_teams_pipelined(lbits, monkeypatch):
    """LC_PIPE bit 2: tile teams overlap steps (team_pipe: per-step mirror slots, super-layer
    tokens, X of a team-slot return read from tile r | j, survivors as per-step bits in HBM).
    With 15-bit tiles a team has more team bits than the pipelined pulls cover, and the
    launch must fall back to the per-step team loop: same answers either way."""
    monkeypatch.setenv("LC_PIPE", "5")
    if lbits:
        monkeypatch.setenv("LC_TILE_LBITS", lbits)
    h, widths, exp = _wide_batch()
    p = _lib.Plan(1, 0, h)
    p.run()
    got = p.results()
    for k in range(h.n_hist):
        _cmp(got, exp[k], k, f"pipelined tile lbits={lbits} w={widths[k]}")
    p.close()


def test_gpu_dense_width_limit_routes_to_grid(monkeypatch):
    """LC_DENSE_MAXW=17 sends the wide histories to the sparse grid kernel: same answers."""
    h, widths, exp = _wide_batch()
    monkeypatch.setenv("LC_DENSE_MAXW", "17")
    p = _lib.Plan(1, 0, h)
    p.run()
    got = p.results()
    assert p.stats()["dense_histories"] == 0
    for k in range(h.n_hist):
        _cmp(got, exp[k], k, f"grid w={widths[k]}")
    p.close()


def test_gpu_dense_edge_histories():
    """Empty, single-op, read-only, all-crashed and fail-only histories through the dense path."""
    ops = [
        [],
        [{"process": 0, "type": "invoke", "f": "read", "value": None},
         {"process": 0, "type": "ok", "f": "read", "value": None}],
        [{"process": 0, "type": "invoke", "f": "read", "value": None},
         {"process": 0, "type": "ok", "f": "read", "value": 3}],
        [{"process": 0, "type": "invoke", "f": "write", "value": 1},
         {"process": 0, "type": "info", "f": "write", "value": 1},
         {"process": 1, "type": "invoke", "f": "cas", "value": [1, 2]},
         {"process": 1, "type": "info", "f": "cas", "value": [1, 2]},
         {"process": 2, "type": "invoke", "f": "read", "value": None},
         {"process": 2, "type": "ok", "f": "read", "value": 2}],
        [{"process": 0, "type": "invoke", "f": "cas", "value": [0, 1]},
         {"process": 0, "type": "fail", "f": "cas", "value": [0, 1]}],
    ]
    h = H.concat([H.encode(o) for o in ops])
    g = _lib.check(1, 0, h)
    exp = oracle.check_many("cas-register", h, n_threads=2)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"edge{k}")
    assert [int(v) for v in g["valid"]] == [1, 1, 0, 1, 1]


@pytest.mark.parametrize("path", ["keys", "grid", "dense"])
def test_gpu_both_kernels_agree_with_oracle(path, monkeypatch):
    """The per-history kernel (keys.hip), the hash-partitioned grid kernel (search.hip) and
    the dense closure tables (dense.hip) must give identical answers on the same batch."""
    monkeypatch.setenv("LC_PATH", path)
    h = synth.gen_register_keys(40, 400, 5, 0.02, config_id=5, invalid_keys=(3, 17, 33))
    g = _lib.check(1, 0, h)
    exp = oracle.check_many("cas-register", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, path)
    c = H.concat([synth.gen_counter(300, 5, 0.005, 7700 + t, invalid=(t % 4 == 0)) for t in range(20)])
    gc = _lib.check(2, 0, c)
    ec = oracle.check_many("counter", c)
    for k in range(c.n_hist):
        _cmp(gc, ec[k], k, path + "-counter")


def test_gpu_keys_capacity_fallback(monkeypatch):
    """Histories that outgrow a workgroup's scratch are re-run by the grid kernel."""
    monkeypatch.setenv("LC_PATH", "keys")
    monkeypatch.setenv("LC_KCAP", "64")
    h = synth.gen_register_keys(32, 600, 5, 0.02, config_id=6, invalid_keys=(4,))
    g = _lib.check(1, 0, h)
    exp = oracle.check_many("cas-register", h)
    assert max(e["max_frontier"] for e in exp) > 64  # the fallback really ran
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, "fallback")


def test_gpu_cell_overflow_buckets(monkeypatch):
    """Cells of 4 entries force most candidates through the per-destination overflow buckets,
    and a 64-entry bucket forces a capacity regrow and re-run: answers must not change."""
    monkeypatch.setenv("LC_PATH", "grid")
    monkeypatch.setenv("LC_CELLCAP", "4")
    monkeypatch.setenv("LC_OVFCAP", "64")
    h = synth.gen_register_keys(12, 500, 5, 0.02, config_id=8, invalid_keys=(5,))
    g = _lib.check(1, 0, h)
    exp = oracle.check_many("cas-register", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, "overflow")


# ---- axis 2: one history, frontier partitioned by config hash (csrc/part.hip) -----------

def _part_row(r):
    return (r["valid"], r["fail_idx"], r["fail_inv"], r["prev_ok"], r["explored"])


def _oracle_part_row(h):
    e = oracle.check_one("cas-register", h)
    bad = e["valid"] == 0
    return (e["valid"], e["fail_idx"] if bad else -1, e["fail_inv_idx"] if bad else -1,
            e["prev_ok_idx"] if bad else -1, e["explored"])


def _part_cases():
    hs = [synth.gen_register_keys(1, 300, 5, 0.02, config_id=7, key0=k) for k in range(4)]
    hs += [synth.gen_register_keys(1, 120, 5, 0.02, config_id=7, key0=k, invalid_keys=(k,))
           for k in (7, 8, 15, 17, 28)]
    hs.append(synth.gen_config("c2", scale=0.1))
    return hs


@pytest.mark.parametrize("device_loop,flow", [(True, "1"), (True, "0"), (False, "1")],
                         ids=["lc_part_run_flow", "lc_part_run_levels", "level_protocol"])
def test_gpu_partitioned_world1_vs_oracle(device_loop, flow, monkeypatch):
    """World 1: lc_part_run's flow form (one work queue per step, no level barriers: the
    default), its level kernel (LC_PART_FLOW=0) and the host-driven level protocol."""
    from lincheck import partition
    monkeypatch.setenv("LC_PART_FLOW", flow)
    for i, h in enumerate(_part_cases()):
        r = partition.check_partitioned(h, device_loop=device_loop)
        assert _part_row(r) == _oracle_part_row(h), (i, r)


def test_gpu_partitioned_matches_dense_on_c2_slice(monkeypatch):
    from lincheck import partition
    h = synth.gen_config("c2", scale=0.3)
    r = partition.check_partitioned(h)  # flow form
    q = partition.check_partitioned(h, device_loop=False)
    monkeypatch.setenv("LC_PART_FLOW", "0")
    lv = partition.check_partitioned(h)  # level kernel
    g = _lib.check(1, 0, h)
    assert (r["valid"], r["explored"]) == (int(g["valid"][0]), int(g["explored"][0]))
    assert (q["valid"], q["explored"]) == (r["valid"], r["explored"])
    assert (q["valid"], q["explored"], q["levels"]) == (lv["valid"], lv["explored"], lv["levels"])


@pytest.mark.parametrize("device_loop,flow", [(True, "1"), (True, "0"), (False, "1")],
                         ids=["lc_part_run_flow", "lc_part_run_levels", "level_protocol"])
def test_gpu_partitioned_capacity_is_unknown(device_loop, flow, monkeypatch):
    from lincheck import partition
    monkeypatch.setenv("LC_PART_FLOW", flow)
    h = synth.gen_config("c2", scale=0.1)
    r = partition.check_partitioned(h, capacity_log2=10, device_loop=device_loop)
    assert r["valid"] == 2 and r["err"] == -7


@pytest.mark.parametrize("flow", ["1", "0"], ids=["flow", "levels"])
def test_gpu_partitioned_run_stage_retry_and_max_steps(flow, monkeypatch):
    """lc_part_run with lists of 2^11: levels whose candidates outgrow the stage make the level
    kernel start over with a 4x stage, a full flow queue reports LC_H_CAPACITY (the oracle's
    answer whenever the sets still fit); max_steps stops early with the explored count of the
    steps run."""
    from lincheck import partition
    monkeypatch.setenv("LC_PART_FLOW", flow)
    for h in _part_cases()[:4]:
        r = partition.check_partitioned(h, capacity_log2=11)
        if r["err"] == 0:
            assert _part_row(r) == _oracle_part_row(h)
    h = _part_cases()[0]
    plan = _lib.PartPlan(h)
    try:
        steps, fail, levels, explored = plan.run(None, 40)
    finally:
        plan.close()
    q = _lib.PartPlan(h)
    try:
        full = partition.search(q, max_steps=40, device_loop=False)
    finally:
        q.close()
    assert (steps, fail, explored) == (40, -1, full["explored"])
    assert levels == (full["levels"] if flow == "0" else 0)


def _pc_row(g):
    return tuple(int(g[k][0]) for k in ("valid", "fail_idx", "fail_inv", "prev_ok", "explored"))


@pytest.mark.parametrize("ranks", [1, 2, 3, 8])
def test_gpu_part_check_in_process_ranks_vs_oracle(ranks):
    """lc_part_check: ONE history, frontier partitioned over in-process ranks (one host thread
    each, candidates pulled by peer/device copies; a JVM caller's single-call axis 2). On a
    1-GPU box the ranks share cuda:0. Bit-exact with the oracle for every rank count."""
    for i, h in enumerate(_part_cases()):
        g = _lib.part_check(h, n_ranks=ranks)
        assert int(g["err"][0]) == 0
        assert _pc_row(g) == _oracle_part_row(h), (ranks, i, g)


def test_gpu_part_check_c2_full_two_ranks_and_capacity():
    """C2 at full size over 2 in-process ranks (22,736 BFS levels through the host exchange):
    the dense path's verdict and explored count; a capacity too small for the frontier gives
    :unknown with LC_H_CAPACITY on every rank count."""
    h = synth.gen_config("c2")
    g = _lib.part_check(h, n_ranks=2)
    d = _lib.check(1, 0, h)
    assert (int(g["valid"][0]), int(g["explored"][0])) == (int(d["valid"][0]), int(d["explored"][0]))
    small = synth.gen_config("c2", scale=0.1)
    for ranks in (1, 2):
        g = _lib.part_check(small, n_ranks=ranks, capacity_log2=10)
        assert int(g["valid"][0]) == 2 and int(g["err"][0]) == -7


def _gpu_part_worker(rank, world, port, q):
    import torch.distributed as tdist
    from lincheck import partition
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, [_part_row(partition.check_partitioned(h, tdist=tdist, device_index=0))
                      for h in _part_cases()[3:]]))
    finally:
        tdist.destroy_process_group()


def test_gpu_partitioned_two_ranks_one_gpu_gloo():
    """Two ranks (processes) on cuda:0, candidates exchanged through gloo: the HIP plan's
    routing, DIRECT returns and per-rank dedup give the oracle's answers."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_part_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=100) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    exp = [_oracle_part_row(h) for h in _part_cases()[3:]]
    for r in range(2):
        assert [tuple(x) for x in got[r]] == exp, (r, got[r], exp)


# ---- offline re-check of a stored history.edn (lincheck.recheck) --------------------------

def test_gpu_recheck_stored_histories(tmp_path):
    from lincheck import recheck
    from lincheck.history import KV
    from test_host import ops_to_edn
    h = synth.gen_register_keys(10, 200, 5, 0.01, config_id=1, invalid_keys=(3, 7))
    ops = []
    for k in range(h.n_hist):
        for o in h.to_ops(k):
            o["value"] = KV(h.keys[k], o["value"])
            ops.append(o)
    ops.sort(key=lambda o: (o["index"], o["value"].key))
    p = tmp_path / "history.edn"
    p.write_text(ops_to_edn(ops))
    res = recheck.recheck(recheck.read_history(str(p), independent=True), "multi-register")
    exp = oracle.check_many("cas-register", h, n_threads=4)
    for k, key in enumerate(h.keys):
        r = res["results"][key]["linear"]
        assert r["valid?"] == {1: True, 0: False}[exp[k]["valid"]], key
        assert r["explored"] == exp[k]["explored"], key
    assert res["valid?"] is (all(e["valid"] == 1 for e in exp))
    assert sorted(res["failures"]) == sorted(h.keys[k] for k in range(h.n_hist) if exp[k]["valid"] != 1)
    # counter workload, one plain history
    c = synth.gen_counter(300, 4, 0.0, 11)
    pc = tmp_path / "counter.edn"
    pc.write_text(ops_to_edn(c.to_ops(0)))
    rc = recheck.main([str(pc), "--workload", "counter"])
    ec = oracle.check_one("counter", c)
    assert rc == (0 if ec["valid"] == 1 else 1)


# ---- the bench's multi-rank protocol (the driver runs it on 2/4/8 GPUs) -------------------

@pytest.mark.parametrize("workload", ["c3", "c5"])
def test_gpu_bench_two_ranks_one_gpu(workload, tmp_path):
    """bench.py under torch.distributed.run with 2 ranks on cuda:0 (gloo; LC_BENCH_DEVICE=0):
    C3's keys split over the ranks (lc_shard_histories), the max-over-ranks time, the summed
    explored count; C5's scan shards with the 5-sum exchange. One JSON line, n_gpus = 2."""
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LC_BENCH_BACKEND="gloo", LC_BENCH_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu", "--workload", workload]
    if workload == "c3":
        cmd += ["--scale", "0.2", "--e2e-reps", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["ms_per_step"] > 0
    if workload == "c3":
        assert out["config"]["histories"] == 200 and out["verdicts"]["0"] == 0
        assert out["configs_explored_per_s"] > 0
    else:
        assert out["verdict"]["bounds_ok"] is True


def test_gpu_bench_gpus_2_launches_its_ranks():
    """plain `python3 bench.py --gpus 2` (no external launcher, as the driver
    runs it) spawns 2 ranks itself; on a 1-GPU box they share cuda:0 and the bench's collectives
    go over gloo. One JSON line with n_gpus = 2 and every key counted once."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LC_BENCH_DEVICE", "LC_BENCH_BACKEND")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu", "--scale", "0.2", "--e2e-reps", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["config"]["histories"] == 200
    assert out["verdicts"]["0"] == 0


# ---- closure tables in HBM (wide.hip): live width 25..35 -------------------

@pytest.mark.parametrize("pipe,grid", [("1", "0"), ("0", "0"), ("1", "8")])
@pytest.mark.parametrize("minw", ["1", "12"])
def test_gpu_wide_tables_vs_oracle(minw, pipe, grid, monkeypatch):
    """The HBM-table kernel, with LC_WIDE_MINW routing every history from that width on to it
    (in production it takes widths 25..35 only): random histories valid and invalid, 16-client
    histories with crashed ops, the low-slot orderings and tiny/empty ones, one launch for all
    of them, bit-exact with the oracle (verdict, failing op, its invocation, :previous-ok,
    explored). LC_WIDE_PIPE=1 (the default) overlaps consecutive steps on the grid, 0 runs one
    step at a time. LC_WIDE_GRID=8 runs the grid on 8 workgroups (the barrier's groups of one)."""
    monkeypatch.setenv("LC_WIDE_MINW", minw)
    monkeypatch.setenv("LC_WIDE_PIPE", pipe)
    monkeypatch.setenv("LC_WIDE_GRID", grid)
    rng = random.Random(5)
    hs = [synth.gen_register(rng.randint(0, 60), rng.randint(1, 8), 0.2, 51000 + t, invalid=(t % 2 == 1))
          for t in range(120)]
    hs += [synth.gen_register(300, 16, 0.01, 52000 + t, invalid=(t % 2 == 1), n_crashed=2 + t) for t in range(4)]
    hs += [_low_slot_rounds(30, 53000 + t, perturb=(t % 2 == 1)) for t in range(6)]
    h = H.concat(hs)
    widths = [_live_width(h, k) for k in range(h.n_hist)]
    g = _lib.check(1, 0, h)
    st = _lib.check_stats()
    n_wide = sum(1 for w in widths if w >= int(minw))
    assert st["wide_histories"] == n_wide and n_wide > 0, (st["wide_histories"], n_wide)
    exp = oracle.check_many("cas-register", h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"wide minw={minw} w={widths[k]}")
    assert any(e["valid"] == 0 for e in exp) and max(widths) >= 17


def test_gpu_wide_tables_match_tile_teams_at_width_24():
    """At the tile teams' limit (width 24: 2.5-2.9 G configs explored) the HBM tables give the
    tile team's explored count and verdict exactly (the crash-ramp histories K = 10, 12)."""
    for k in (10, 12):
        h = synth.gen_register(2000, 16, 0.002, 0x5EED4000 + k, n_crashed=k)
        assert _live_width(h, 0) == 24
        a = _lib.check(1, 0, h)
        assert _lib.check_stats()["wide_histories"] == 0
        os.environ["LC_WIDE_MINW"] = "24"
        try:
            b = _lib.check(1, 0, h)
            assert _lib.check_stats()["wide_histories"] == 1
        finally:
            del os.environ["LC_WIDE_MINW"]
        for key in ("valid", "fail_idx", "explored"):
            assert int(a[key][0]) == int(b[key][0]), (k, key, a[key][0], b[key][0])
        assert int(a["explored"][0]) > 2_000_000_000


def _with_never_ops(h, n):
    """h with n more calls pending for its whole length: cas 9 -> 8 by n extra processes,
    invoked first and completed :info last. The register never holds 9, so no config ever
    linearizes them: the verdict and the explored count are h's, the live width is h's + n."""
    m = n + int(h.n) + n
    proc = np.concatenate([10000 + np.arange(n), h.process, 10000 + np.arange(n)]).astype(np.int32)
    typ = np.concatenate([np.zeros(n), h.type, np.full(n, 3)]).astype(np.int8)
    f = np.concatenate([np.full(n, 2), h.f, np.full(n, 2)]).astype(np.int8)
    v0 = np.concatenate([np.full(n, 9), h.v0, np.full(n, 9)]).astype(np.int64)
    v1 = np.concatenate([np.full(n, 8), h.v1, np.full(n, 8)]).astype(np.int64)
    vf = np.concatenate([np.full(n, H.V_PAIR), h.vflags, np.full(n, H.V_PAIR)]).astype(np.int8)
    return H.from_columns(np.arange(m), proc, typ, f, v0, v1, vf)


def test_gpu_wide_tables_past_the_tile_teams():
    """Widths 25..31 against the oracle: 400-op histories of 14 clients plus up to 18 calls that
    are pending throughout and can never apply (so the oracle's frontier stays small while the
    tables are 2^22..2^27 words), valid and with a read of a value never written; then the crash
    ramp's width-27 history (K = 13; the grid kernel did not finish it in 3 minutes)."""
    for n, bad, seed in ((11, False, 54011), (12, True, 54012), (14, False, 54014), (16, True, 54016),
                         (18, False, 54000)):  # (the last one: width 31, the limit)
        base = synth.gen_register(400, 14, 0.0, seed)
        if bad:  # a read of a value the register never holds (7; the domain is 0..4)
            reads = [i for i in range(base.n) if base.type[i] == 1 and base.f[i] == 0 and base.vflags[i] == H.V_SCALAR]
            v0 = base.v0.copy()
            v0[reads[len(reads) // 2]] = 7
            base = H.from_columns(base.index, base.process, base.type, base.f, v0, base.v1, base.vflags)
        h = _with_never_ops(base, n)
        w = _live_width(h, 0)
        assert 24 < w <= 31, w
        g = _lib.check(1, 0, h)
        assert _lib.check_stats()["wide_histories"] == 1
        e = oracle.check_one("cas-register", h)
        assert e["valid"] == (0 if bad else 1)
        _cmp(g, e, 0, f"wide w={w}")
        assert int(g["explored"][0]) == oracle.check_one("cas-register", base)["explored"]
        if bad:  # the failure report straight from the HBM tables, as sets
            _check_configs_vs_oracle(h, f"wide w={w}")
    h = synth.gen_register(2000, 16, 0.002, 0x5EED4000 + 13, n_crashed=13)
    assert _live_width(h, 0) == 27
    g = _lib.check(1, 0, h)
    assert _lib.check_stats()["wide_histories"] == 1
    assert int(g["valid"][0]) == 1 and int(g["explored"][0]) > 0


def _check_configs_vs_oracle(h, what, k=1 << 12):
    """lc_failure_configs of history 0 of the last check against the oracle's pre-failure frontier:
    the configs as a set, each config's :last-op, the newest, the pending ops."""
    e = oracle.check_one("cas-register", h, with_configs=True)
    assert e["valid"] == 0, what
    cfgs, pending, lasts, newest = _lib.failure_configs(0, k, with_last=True)
    assert sorted(pending) == sorted(e["pending_inv_idx"]), what
    assert set(cfgs) == e["fail_configs"] and len(cfgs) == len(e["fail_configs"]), what
    for c, last in zip(cfgs, lasts):
        assert last == e["fail_last_op"][c], (what, c, last, e["fail_last_op"][c])
    assert newest == max(e["fail_last_op"].values()), what
    return sum(1 for x in lasts if x != e["prev_ok_idx"])


@pytest.mark.parametrize("pipe", ["1", "0"])
def test_gpu_wide_failure_configs_match_oracle(pipe, monkeypatch):
    """failure reports from the HBM tables (wide.hip: a re-run stopped before
    the failing RETURN, the frontier dumped from the table, each config's :last-op walked back
    through the final tables, re-running to earlier stops for long walks). Every history forced
    onto the tables (LC_WIDE_MINW=1), both table layouts (pipelined: ranked; one step at a
    time: natural), against the oracle: configs as sets, per-config :last-op, the newest, and
    the grid kernel's report (LC_WIDE_CONFIGS=0) on the same history."""
    monkeypatch.setenv("LC_WIDE_MINW", "1")
    monkeypatch.setenv("LC_WIDE_PIPE", pipe)
    found = carried = 0
    for t in range(30):
        h = synth.gen_register(80, 4, 0.1, 9000 + t, invalid=True, n_crashed=t % 3)
        g = _lib.check(1, 0, h)
        assert _lib.check_stats()["wide_histories"] == 1
        e = oracle.check_one("cas-register", h)
        assert int(g["valid"][0]) == e["valid"]
        if e["valid"] != 0:
            continue
        carried += _check_configs_vs_oracle(h, f"t={t}")
        found += 1
        if t % 5 == 0:  # the same report through the grid kernel's tagged re-run
            a = _lib.failure_configs(0, 1 << 12, with_last=True)
            monkeypatch.setenv("LC_WIDE_CONFIGS", "0")
            b = _lib.failure_configs(0, 1 << 12, with_last=True)
            monkeypatch.delenv("LC_WIDE_CONFIGS")
            assert a == b, t
    assert found > 5 and carried > 0


def test_gpu_wide_tables_past_31_slots():
    """r4: the HBM tables up to live width 35 (2 x 2^32 words = 64 GiB),
    stream headers with 64-bit live masks. Small bases with up to 32 calls pending throughout
    that can never apply (so the oracle stays fast while the tables reach 2^29..2^32 words per
    step), valid and with a read of a value never written, against the oracle."""
    for base_ops, clients, n, bad, seed in ((60, 4, 28, False, 57000), (60, 4, 29, True, 57001),
                                            (40, 3, 31, False, 57002), (30, 3, 32, True, 57003)):
        base = synth.gen_register(base_ops, clients, 0.0, seed)
        if bad:
            reads = [i for i in range(base.n) if base.type[i] == 1 and base.f[i] == 0 and base.vflags[i] == H.V_SCALAR]
            if reads:
                v0 = base.v0.copy()
                v0[reads[len(reads) // 2]] = 7
                base = H.from_columns(base.index, base.process, base.type, base.f, v0, base.v1, base.vflags)
        h = _with_never_ops(base, n)
        w = _live_width(h, 0)
        assert 31 < w <= 35, w
        g = _lib.check(1, 0, h)
        assert _lib.check_stats()["wide_histories"] == 1, w
        e = oracle.check_one("cas-register", h)
        _cmp(g, e, 0, f"wide w={w}")
        assert int(g["explored"][0]) == oracle.check_one("cas-register", base)["explored"]
        if bad and e["valid"] == 0:
            _check_configs_vs_oracle(h, f"wide w={w}")


def _read_never_written(h, at_frac):
    """h with its first :ok scalar read from entry at_frac * n on returning 7, a value the
    generator never writes (its domain is 0..4): invalid from that read on."""
    reads = [i for i in range(int(at_frac * h.n), h.n)
             if h.type[i] == 1 and h.f[i] == 0 and h.vflags[i] == H.V_SCALAR]
    v0 = h.v0.copy()
    v0[reads[0]] = 7
    return H.from_columns(h.index, h.process, h.type, h.f, v0, h.v1, h.vflags)


@pytest.mark.parametrize("split", ["1", "2", "3"])
def test_gpu_wide_slabs_vs_oracle(split, monkeypatch):
    """the HBM tables split by their top `split` hi bits into 2^split slabs
    (each ranked over its own hi bits; pulls over a split bit read the neighbouring slab), forced
    with LC_WIDE_SPLIT on every history from width 12 on: random valid and invalid histories and
    16-client ones with crashed ops against the oracle, and one failure report as sets."""
    monkeypatch.setenv("LC_WIDE_MINW", "12")
    monkeypatch.setenv("LC_WIDE_SPLIT", split)
    hs = [synth.gen_register(300, 16, 0.01, 52100 + t, n_crashed=2 + t) for t in range(6)]
    hs += [synth.gen_register(200, 12, 0.05, 52200 + t) for t in range(6)]
    h = H.concat([_read_never_written(x, 0.3 + 0.1 * (t % 5)) if t % 2 else x for t, x in enumerate(hs)])
    widths = [_live_width(h, k) for k in range(h.n_hist)]
    g = _lib.check(1, 0, h)
    st = _lib.check_stats()
    assert st["wide_histories"] == sum(1 for w in widths if w >= 12) > 0
    assert int(st["wide_slabs"]) == 1 << int(split)
    exp = oracle.check_many("cas-register", h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"slabs split={split} w={widths[k]}")
    bad = [k for k in range(h.n_hist) if exp[k]["valid"] == 0 and widths[k] >= 12]
    assert bad
    one = h.select([min(bad, key=lambda k: exp[k]["explored"])])
    g1 = _lib.check(1, 0, one)
    assert int(g1["valid"][0]) == 0 and int(_lib.check_stats()["wide_slabs"]) == 1 << int(split)
    _check_configs_vs_oracle(one, f"slabs split={split}")


def test_gpu_wide_slabs_match_one_table_on_the_crash_ramp():
    """The slab split (2, 4, 8 slabs: the table's rank split multiplexed on one device) gives the
    single table's verdict, failing op and explored count on the crash ramp's real wide frontiers
    (K = 13..18: widths 27..33, 7 G to 390 G configs)."""
    for k in (13, 14, 16, 18):
        h = synth.gen_register(2000, 16, 0.002, 0x5EED4000 + k, n_crashed=k)
        a = _lib.check(1, 0, h)
        st = _lib.check_stats()
        assert st["wide_histories"] == 1 and int(st["wide_slabs"]) == 1, (k, st["wide_slabs"])
        for split in ("1", "2", "3"):
            os.environ["LC_WIDE_SPLIT"] = split
            try:
                b = _lib.check(1, 0, h)
                st = _lib.check_stats()
            finally:
                del os.environ["LC_WIDE_SPLIT"]
            assert st["wide_histories"] == 1 and int(st["wide_slabs"]) == 1 << int(split)
            for key in ("valid", "fail_idx", "fail_inv", "prev_ok", "explored"):
                assert int(a[key][0]) == int(b[key][0]), (k, split, key, a[key][0], b[key][0])


def test_gpu_wide_tables_at_width_36():
    """r5: live width 36 (2 x 2^33 words = 128 GiB, two slabs of 2^32 words per table: a slab's
    index is 32-bit): a 12-op base with 34 calls pending throughout that can never apply, valid
    and with a read of a value never written, against the oracle."""
    for n, bad, seed in ((34, False, 57100), (34, True, 57101)):
        base = synth.gen_register(12, 2, 0.0, seed)
        if bad:
            reads = [i for i in range(base.n) if base.type[i] == 1 and base.f[i] == 0 and base.vflags[i] == H.V_SCALAR]
            assert reads
            v0 = base.v0.copy()
            v0[reads[-1]] = 7
            base = H.from_columns(base.index, base.process, base.type, base.f, v0, base.v1, base.vflags)
        h = _with_never_ops(base, n)
        w = _live_width(h, 0)
        assert w == 36, w
        g = _lib.check(1, 0, h)
        st = _lib.check_stats()
        assert st["wide_histories"] == 1 and int(st["wide_slabs"]) == 2, (w, st["wide_slabs"])
        e = oracle.check_one("cas-register", h)
        assert e["valid"] == (0 if bad else 1)
        _cmp(g, e, 0, f"wide w={w}")
        assert int(g["explored"][0]) == oracle.check_one("cas-register", base)["explored"]
        if bad:
            _check_configs_vs_oracle(h, f"wide w={w}")


def test_gpu_wide_watchdog_abort_is_unknown(monkeypatch):
    """when the HBM tables' grid barrier watchdog fires (its abort word forced here
    with LC_WIDE_FORCE_ABORT=1, as a fired watchdog leaves it) the call still succeeds: the wide
    histories it did not finish are :unknown with LC_H_ABORTED, every other history of the call
    keeps its answer."""
    monkeypatch.setenv("LC_WIDE_MINW", "12")
    monkeypatch.setenv("LC_WIDE_FORCE_ABORT", "1")
    narrow = [synth.gen_register(200, 4, 0.01, 56000 + t, invalid=(t % 2 == 1)) for t in range(6)]
    wide = synth.gen_register(400, 16, 0.01, 56100, n_crashed=2)
    h = H.concat(narrow + [wide])
    assert _live_width(h, h.n_hist - 1) >= 12 and all(_live_width(h, k) < 12 for k in range(len(narrow)))
    g = _lib.check(1, 0, h)
    assert _lib.check_stats()["wide_histories"] == 1
    last = h.n_hist - 1
    assert int(g["valid"][last]) == 2 and int(g["err"][last]) == -8
    exp = oracle.check_many("cas-register", h.select(list(range(len(narrow)))))
    for k in range(len(narrow)):
        _cmp(g, exp[k], k, "beside an aborted wide history")
    monkeypatch.delenv("LC_WIDE_FORCE_ABORT")
    g2 = _lib.check(1, 0, h)  # the next call runs normally
    assert int(g2["valid"][last]) == oracle.check_one("cas-register", h.select([last]))["valid"]


@pytest.mark.parametrize("pipe", ["1", "0"])
def test_gpu_wide_watchdog_real_stall(pipe, monkeypatch):
    """VERDICT r4 item 8 / ADVICE r4: a grid barrier that REALLY stalls. Workgroup 3 skips its
    barrier arrival at the start of the second wide history (LC_WIDE_STALL=1:3), so no workgroup
    can pass that barrier and the 200 ms watchdog (wide.hip wide_sync) ends the launch. The first
    wide history finished before the stall: its verdict AND explored count equal the oracle's
    (the status is written only after every workgroup added its count). The stalled history and
    the ones after it are :unknown (LC_H_ABORTED), the narrow histories keep their answers, and
    the next call runs normally."""
    monkeypatch.setenv("LC_WIDE_MINW", "12")
    monkeypatch.setenv("LC_WIDE_PIPE", pipe)
    monkeypatch.setenv("LC_WIDE_WATCHDOG_MS", "200")
    monkeypatch.setenv("LC_WIDE_STALL", "1:3")
    narrow = [synth.gen_register(200, 4, 0.01, 56200 + t, invalid=(t % 2 == 1)) for t in range(6)]
    wide = [synth.gen_register(400, 16, 0.01, 56300 + t, n_crashed=2, invalid=(t == 0)) for t in range(3)]
    h = H.concat(narrow + wide)
    nw = len(narrow)
    assert all(_live_width(h, k) >= 12 for k in range(nw, h.n_hist))
    assert all(_live_width(h, k) < 12 for k in range(nw))
    exp = oracle.check_many("cas-register", h)
    g = _lib.check(1, 0, h)
    assert _lib.check_stats()["wide_histories"] == 3
    for k in range(nw):
        _cmp(g, exp[k], k, "beside a stalled wide launch")
    decided = [k for k in range(nw, h.n_hist) if int(g["err"][k]) != -8]
    aborted = [k for k in range(nw, h.n_hist) if int(g["err"][k]) == -8]
    assert len(decided) == 1 and len(aborted) == 2, (decided, aborted, g["err"][nw:])
    for k in decided:
        _cmp(g, exp[k], k, "finished before the stall")
    for k in aborted:
        assert int(g["valid"][k]) == 2
    monkeypatch.delenv("LC_WIDE_STALL")
    g2 = _lib.check(1, 0, h)  # a clean next call
    for k in range(h.n_hist):
        _cmp(g2, exp[k], k, "after the stall")


def test_gpu_fuzz_register_and_counter_vs_oracle():
    """Random histories of both models, one lc_check per model (the batch planner sees them all
    together): 1-8 clients, 1-400 ops, 0-4 crashed writes/cas, :info on any op, valid and
    perturbed, plus counters; bit-exact with the oracle. LC_FUZZ_N scales the register count
    (default 200; r3ao ran 2000 on the GPU box, `profiles/r3ao`)."""
    n = int(os.environ.get("LC_FUZZ_N", "200"))
    rng = random.Random(71)
    hs = []
    for t in range(n):
        hs.append(synth.gen_register(rng.randint(1, 400), rng.randint(1, 8), rng.choice([0.0, 0.01, 0.05]),
                                     900000 + t, invalid=(t % 2 == 1),
                                     n_crashed=rng.choice([None, 0, 1, 2, 4])))
    h = H.concat(hs)
    g = _lib.check(1, 0, h)
    exp = oracle.check_many("cas-register", h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, "fuzz register")
    assert 0 < sum(e["valid"] == 0 for e in exp) < len(exp)
    cs = [synth.gen_counter(rng.randint(1, 300), rng.randint(1, 8), 0.02, 910000 + t, invalid=(t % 3 == 2))
          for t in range(max(20, n // 5))]
    hc = H.concat(cs)
    gc = _lib.check(2, 0, hc)
    expc = oracle.check_many("counter", hc, n_threads=8)
    for k in range(hc.n_hist):
        _cmp(gc, expc[k], k, "fuzz counter")


def test_gpu_fuzz_wide_register_vs_oracle():
    """Wider random register histories in one lc_check: 12-16 clients, 100-400 ops, 0-5 crashed
    writes/cas (live widths into the BLOCK, MID and tile-team classes, so the team planner's
    12-slot tiles are in play), valid and perturbed; bit-exact with the oracle. LC_FUZZ_WIDE_N
    scales it (default 60; r3ap ran 300 on the GPU box, `profiles/r3ap`)."""
    n = int(os.environ.get("LC_FUZZ_WIDE_N", "60"))
    rng = random.Random(73)
    hs = [synth.gen_register(rng.randint(100, 400), rng.randint(12, 16), rng.choice([0.0, 0.01]), 930000 + t,
                             invalid=(t % 2 == 1), n_crashed=rng.choice([0, 2, 4, 5])) for t in range(n)]
    h = H.concat(hs)
    widths = [_live_width(h, k) for k in range(h.n_hist)]
    g = _lib.check(1, 0, h)
    st = _lib.check_stats()
    exp = oracle.check_many("cas-register", h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"fuzz wide w={widths[k]}")
    assert st["dense_histories"] == h.n_hist and max(widths) >= 17
    assert any(e["valid"] == 0 for e in exp)
