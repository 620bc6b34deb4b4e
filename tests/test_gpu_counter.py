"""GPU parity tests of the counter workload's exact search: the counter
closure tables (csrc/ctab.hip) through the C-ABI against the CPU oracle and the
oracle-pinned fixtures of tests/golden/counter_*_oracle.json (tests/golden/pin_counter.py).

The reference checks a counter run as ONE whole-history knossos.linear search with CounterModel
(src/jepsen/jgroups/workload/counter.clj:100-137); these tests hold the GPU's answer for that
search — verdict, failing :index triple and explored count — to the oracle's at C2's shape
(1 key x 5k ops, 16 clients), with crashed ops, and at C5's low-crash exact-search size."""
import json
import os
import random
import sys

import numpy as np
import pytest

import oracle
from lincheck import _lib, history as H, synth

pytestmark = pytest.mark.gpu
GOLD_DIR = os.path.join(os.path.dirname(__file__), "golden")


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


def _fixture(name):
    p = os.path.join(GOLD_DIR, f"counter_{name}_oracle.json")
    if not os.path.exists(p):
        pytest.skip(f"{p} not pinned yet (tests/golden/pin_counter.py {name})")
    return json.load(open(p))


def _live_width(h, k):
    """Most calls pending at once in history k (crashed ones stay pending; :fail ones never enter)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    from crash_ramp import width_of
    return width_of(h.select([k]))


def _ctab_count():
    return int(_lib.check_stats(0)["ctab_histories"])


def _mixed_counters(n, seed0, max_ops=300, max_clients=16, max_crash=3):
    rng = random.Random(seed0)
    hs = []
    for t in range(n):
        # exactly k crashed ops (p_info then only fails reads): each crashed op stays pending for
        # good and can double the frontier, so the oracle's time is kept to seconds
        hs.append(synth.gen_counter(rng.randint(1, max_ops), rng.randint(1, max_clients),
                                    rng.choice([0.0, 0.05, 0.1]), seed0 * 1000 + t,
                                    invalid=(t % 3 == 2), n_crashed=rng.randint(0, max_crash)))
    return H.concat(hs)


@pytest.mark.parametrize("pipe", ["1", "0"])
def test_gpu_ctab_random_vs_oracle(pipe, monkeypatch):
    """Many counter histories in one lc_check (one per workgroup, dequeued heaviest first):
    1-16 clients, crashed ops, :fail reads, perturbed reads; double-buffered tables and the
    single-table form (LC_CTAB_PIPE=0, a step two super-layers after its predecessor)."""
    monkeypatch.setenv("LC_CTAB_PIPE", pipe)
    h = _mixed_counters(240, 31)
    g = _lib.check(2, 0, h)
    assert _ctab_count() == h.n_hist
    exp = oracle.check_many("counter", h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"ctab pipe={pipe}")
    assert any(e["valid"] == 0 for e in exp) and any(e["valid"] == 1 for e in exp)


@pytest.mark.parametrize("T,pipe", [("1", "3"), ("2", "3"), ("3", "3"), ("4", "3"), ("2", "0")])
def test_gpu_ctab_teams_vs_oracle(T, pipe, monkeypatch):
    """counter tile teams (ctab_team_kernel: one history's table split over
    2^T workgroups by its top T slots, mirrors in HBM between tiles) forced from
    width 9 on, T = 1..4, double- and single-buffered tiles: bit-exact with the oracle on random
    histories (crashed ops, :fail reads, perturbed reads) and with the one-workgroup kernel."""
    monkeypatch.setenv("LC_CTAB_TEAM_MINW", "9")
    monkeypatch.setenv("LC_CTAB_TEAM_T", T)
    monkeypatch.setenv("LC_CTAB_PIPE", pipe)
    h = _mixed_counters(60, 7100 + int(T) + 10 * int(pipe), max_ops=300, max_clients=16, max_crash=3)
    g = _lib.check(2, 0, h)
    assert _ctab_count() == h.n_hist
    exp = oracle.check_many("counter", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"team T={T}")
    monkeypatch.setenv("LC_CTAB_TEAM", "0")
    g1 = _lib.check(2, 0, h)
    for key in ("valid", "fail_idx", "explored"):
        assert np.array_equal(g[key], g1[key]), key


def test_gpu_ctab_matches_grid_kernel(monkeypatch):
    """The same batch on the closure tables and on the grid kernel (LC_CTAB_MAXW=0)."""
    h = _mixed_counters(60, 47, max_ops=200)
    a = _lib.check(2, 0, h)
    assert _ctab_count() == h.n_hist
    monkeypatch.setenv("LC_CTAB_MAXW", "0")
    b = _lib.check(2, 0, h)
    assert _ctab_count() == 0
    for key in ("valid", "fail_idx", "fail_inv", "prev_ok", "explored", "err"):
        assert np.array_equal(a[key], b[key]), key


@pytest.mark.parametrize("init", [0, 7, -123456, 2**40])
def test_gpu_ctab_init_value(init):
    """Requirements are relative to the initial value (counter.clj:133: (CounterModel. 0); the
    C-ABI takes any init_value)."""
    hs = [synth.gen_counter(150, 8, 0.02, 5100 + t, invalid=(t % 2 == 1)) for t in range(6)]
    h = H.concat(hs)
    g = _lib.check(2, init, h)
    for k in range(h.n_hist):
        _cmp(g, oracle.check_one("counter", h.select([k]), init_value=init), k, f"init={init}")


@pytest.mark.parametrize("team", ["1", "0"])
def test_gpu_ctab_wide_deltas_and_widths_route_to_grid(team, monkeypatch):
    """Histories the tables do not take (|delta| > 10; wider than 20 live slots without tile
    teams, LC_CTAB_TEAM=0) go to the grid kernel in the same call; every answer still matches
    the oracle."""
    monkeypatch.setenv("LC_CTAB_TEAM", team)
    big = synth.gen_counter(120, 5, 0.0, 77)
    big.v0 = np.where((big.f == 3) & (big.vflags == 1), big.v0 * 20, big.v0)  # adds of 0..80
    big = H.from_columns(big.index, big.process, big.type, big.f, big.v0, big.v1, big.vflags)
    wide = synth.gen_counter(160, 16, 0.0, 78, n_crashed=6, crash_span=0.1)
    ok = synth.gen_counter(200, 8, 0.0, 79)
    h = H.concat([big, wide, ok])
    g = _lib.check(2, 0, h)
    exp = oracle.check_many("counter", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, "routing")
    assert _ctab_count() >= 1


def test_gpu_ctab_edge_histories():
    """Empty, invoke-only, one op, a read of nil, decr-and-get and a *-and-get that crashed."""
    E = lambda *ev: H.encode([dict(zip(("process", "type", "f", "value"), e)) for e in ev])  # noqa: E731
    cases = [
        E(),
        E((0, "invoke", "add", 3)),
        E((0, "invoke", "add", 3), (0, "ok", "add", 3)),
        E((0, "invoke", "read", None), (0, "ok", "read", None)),
        E((0, "invoke", "decr-and-get", 2), (0, "ok", "decr-and-get", [2, -2]),
          (1, "invoke", "read", None), (1, "ok", "read", -2)),
        E((0, "invoke", "add-and-get", 4), (0, "info", "add-and-get", 4),
          (1, "invoke", "read", None), (1, "ok", "read", 4)),
        E((0, "invoke", "add-and-get", 4), (0, "info", "add-and-get", 4),
          (1, "invoke", "read", None), (1, "ok", "read", 3)),
        E((0, "invoke", "add", 1), (1, "invoke", "read", None), (1, "ok", "read", 2), (0, "ok", "add", 1)),
    ]
    h = H.concat(cases)
    g = _lib.check(2, 0, h)
    exp = oracle.check_many("counter", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"edge {k}")


def test_gpu_ctab_c2c_full_size_vs_fixture():
    """C2's shape as a counter (1 key x 5k ops, 16 clients) at full size, against the oracle's
    pinned answer (tests/golden/counter_c2c_oracle.json)."""
    fx = _fixture("c2c")
    h = synth.gen_config("c2c")
    assert h.n == fx["n_entries"] and h.n_ops() == fx["n_ops"]
    g = _lib.check(2, 0, h)
    assert _ctab_count() == 1
    assert int(g["valid"][0]) == fx["valid"] and int(g["fail_idx"][0]) == fx["fail_idx"]
    assert int(g["explored"][0]) == fx["explored"]


def test_gpu_ctab_c2c_crashed_vs_fixture():
    """The same shape with 4 crashed ops pending through the rest of the history (width 20)."""
    fx = _fixture("c2c4")
    h = synth.gen_counter(5000, 16, 0.0, 12345, n_crashed=4)
    assert h.n == fx["n_entries"]
    g = _lib.check(2, 0, h)
    assert _ctab_count() == 1
    assert int(g["valid"][0]) == fx["valid"] and int(g["explored"][0]) == fx["explored"]


def test_gpu_ctab_c2c_perturbed_prefixes_vs_oracle():
    """C2c perturbed at random reads (invalid): the failing :index triple and explored count of
    every prefix the oracle finishes quickly."""
    for seed in range(3):
        h = synth.gen_counter(2500, 16, 0.0, 6100 + seed, invalid=True)
        g = _lib.check(2, 0, h)
        _cmp(g, oracle.check_one("counter", h), 0, f"c2c-invalid-{seed}")


def test_gpu_ctab_c5x_full_size_vs_fixture():
    """C5's low-crash exact-search variant (1M ops, 16 clients, 4 crashed ops live throughout)
    at full size, against the oracle's pinned answer (hours on one core)."""
    fx = _fixture("c5x")
    h = synth.gen_config("c5x")
    assert h.n == fx["n_entries"] and h.n_ops() == fx["n_ops"]
    g = _lib.check(2, 0, h)
    assert _ctab_count() == 1
    assert int(g["valid"][0]) == fx["valid"] and int(g["explored"][0]) == fx["explored"]


def _counter_ramp():
    """Counter histories with K crashed ops (each a slot live for good): live widths 21..24, past
    one workgroup's LDS table (20), each a few seconds of the oracle."""
    hs = [synth.gen_counter(ops, cl, 0.0, 777 + k, n_crashed=k)
          for ops, cl, k in ((400, 16, 8), (300, 16, 9), (300, 16, 7), (400, 14, 8), (350, 16, 9))]
    hs += [synth.gen_counter(400, 16, 0.0, 7800 + t, n_crashed=7, invalid=True) for t in range(3)]
    return H.concat(hs)


def test_gpu_ctab_teams_past_20_slots_vs_oracle():
    """counters wider than one workgroup's table (live width 21..24, the step
    header's limit) on tile teams of 2^T workgroups (T = width - 15: 64 tiles at 24), bit-exact
    with the oracle (verdict, failing :index triple, explored); no grid-kernel fallback."""
    h = _counter_ramp()
    widths = [_live_width(h, k) for k in range(h.n_hist)]
    assert max(widths) >= 23 and min(widths) >= 21, widths
    assert max(widths) <= 24, widths
    g = _lib.check(2, 0, h)
    st = _lib.check_stats()
    assert int(st["ctab_team_histories"]) == h.n_hist and int(st["ctab_histories"]) == h.n_hist, st
    exp = oracle.check_many("counter", h)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"counter width {widths[k]}")
    assert any(e["valid"] == 0 for e in exp) and any(e["valid"] == 1 for e in exp)


# ---- counters on the HBM tables (wctr_pipe_kernel): live width 25..36 --------

@pytest.mark.parametrize("grid", ["0", "8"])
def test_gpu_wctr_vs_oracle(grid, monkeypatch):
    """the counter closure tables in HBM (one ranked table of 2^(L-6) words,
    the grid-wide pipelined schedule of wide.hip, ctab's EQ gates), with LC_WCTR_MINW=1 routing
    every counter to them (in production they take widths 25..36 only): random histories with
    crashed ops, :fail reads and perturbed reads, bit-exact with the oracle (verdict, failing
    :index triple, explored). LC_WIDE_GRID=8 runs the grid on 8 workgroups."""
    monkeypatch.setenv("LC_WCTR_MINW", "1")
    monkeypatch.setenv("LC_WIDE_GRID", grid)
    h = _mixed_counters(80, 7300 + int(grid), max_ops=250, max_clients=16, max_crash=4)
    g = _lib.check(2, 0, h)
    st = _lib.check_stats()
    assert int(st["wide_histories"]) == h.n_hist, st
    exp = oracle.check_many("counter", h, n_threads=8)
    for k in range(h.n_hist):
        _cmp(g, exp[k], k, f"wctr grid={grid}")
    assert any(e["valid"] == 0 for e in exp) and any(e["valid"] == 1 for e in exp)


@pytest.mark.parametrize("init", [0, -123456])
def test_gpu_wctr_matches_ctab(init, monkeypatch):
    """The same counters on the HBM tables (LC_WCTR_MINW=1) and on the LDS tables / tile teams."""
    h = H.concat([synth.gen_counter(400, 16, 0.0, 7400 + t, n_crashed=t % 5, invalid=(t % 3 == 1)) for t in range(12)])
    a = _lib.check(2, init, h)
    assert int(_lib.check_stats()["wide_histories"]) == 0
    monkeypatch.setenv("LC_WCTR_MINW", "1")
    b = _lib.check(2, init, h)
    assert int(_lib.check_stats()["wide_histories"]) == h.n_hist
    for key in ("valid", "fail_idx", "fail_inv", "prev_ok", "explored", "err"):
        assert np.array_equal(a[key], b[key]), key


def test_gpu_wctr_counter_ramp_vs_oracle():
    """The counter crash ramp past the tile teams (K = 10, 12, 14: live width 25, 27, 29; the
    grid kernel's range until r5) on the HBM tables, against the oracle's explored counts and
    verdicts (tests/golden/counter_ramp_oracle.json, from tools/crash_ramp.py --model counter)."""
    fx = json.load(open(os.path.join(GOLD_DIR, "counter_ramp_oracle.json")))
    cases = {c["crashed"]: c for c in fx["cases"]}
    for k in (10, 12, 14):
        h = synth.gen_counter(2000, 16, 0.0, 0x5EED4000 + 0x100 + k, n_crashed=k, crash_span=0.2)
        assert _live_width(h, 0) == cases[k]["width"]
        g = _lib.check(2, 0, h)
        st = _lib.check_stats()
        assert int(st["wide_histories"]) == 1, (k, st)
        assert (int(g["valid"][0]), int(g["explored"][0])) == (cases[k]["valid"], cases[k]["explored"]), k


def test_gpu_wctr_widths_36_38_vs_oracle():
    """The widest counter tables (36 and 38 live slots; 2 x 2^32 words at 38): a 40-op base with up to 32 calls that
    are pending throughout and can never apply (add-and-get [1 10^9], completed :info at the end:
    a vector value is checked even for :info, counter.clj:114-119, and no config reaches 10^9 - 1),
    valid and invalid, against the oracle; the explored count is the base's."""
    for bad, seed, width in ((False, 7500, 36), (True, 7501, 36), (False, 7502, 38), (True, 7503, 38)):
        base = synth.gen_counter(40, 6, 0.0, seed, invalid=bad)
        n = width - _live_width(base, 0)
        # the never-ops invoked in two groups around the base's first completion (a step holds at
        # most WCTR_MAX_NINV = 30 invocations), completed :info at the end
        c0 = int(np.nonzero(np.asarray(base.type) != 0)[0][0]) + 1
        half = n // 2
        seg = lambda a, b: np.arange(a, b)  # noqa: E731
        rows = [("x", seg(0, half)), ("b", seg(0, c0)), ("x", seg(half, n)), ("b", seg(c0, int(base.n))), ("y", seg(0, n))]
        cols = {k: [] for k in ("proc", "typ", "f", "v0", "v1", "vf")}
        for kind, ix in rows:
            if kind == "b":
                vals = (base.process[ix], base.type[ix], base.f[ix], base.v0[ix], base.v1[ix], base.vflags[ix])
            else:  # add-and-get [1 10^9]: invoked ("x"), completed :info ("y")
                vals = (20000 + ix, np.full(len(ix), 0 if kind == "x" else 3), np.full(len(ix), 5),
                        np.full(len(ix), 1), np.full(len(ix), 10 ** 9), np.full(len(ix), H.V_PAIR))
            for key, v in zip(cols, vals):
                cols[key].append(np.asarray(v))
        c = {k: np.concatenate(v) for k, v in cols.items()}
        h = H.from_columns(np.arange(len(c["proc"])), c["proc"].astype(np.int32), c["typ"].astype(np.int8),
                           c["f"].astype(np.int8), c["v0"].astype(np.int64), c["v1"].astype(np.int64),
                           c["vf"].astype(np.int8))
        w = _live_width(h, 0)
        assert w == width, w
        g = _lib.check(2, 0, h)
        assert int(_lib.check_stats()["wide_histories"]) == 1
        e = oracle.check_one("counter", h)
        _cmp(g, e, 0, f"wctr w={w} bad={bad}")
        assert int(g["explored"][0]) == oracle.check_one("counter", base)["explored"]
        if bad:  # the failure report from the width-36/38 tables
            _configs_vs_oracle(h, f"wctr w={w}")


def _configs_vs_oracle(h, what):
    e = oracle.check_one("counter", h, with_configs=True)
    assert e["valid"] == 0, what
    cfgs, pending, lasts, newest = _lib.failure_configs(0, 1 << 12, with_last=True)
    assert sorted(pending) == sorted(e["pending_inv_idx"]), what
    assert set(cfgs) == e["fail_configs"] and len(cfgs) == len(e["fail_configs"]), what
    for c, last in zip(cfgs, lasts):
        assert last == e["fail_last_op"][c], (what, c, last, e["fail_last_op"][c])
    assert newest == max(e["fail_last_op"].values()), what
    return sum(1 for x in lasts if x != e["prev_ok_idx"])


def test_gpu_wctr_failure_configs_match_oracle(monkeypatch):
    """Failure reports straight from the HBM counter tables (a re-run stopped before the failing
    RETURN, the frontier dumped as masks, each config's :last-op walked back with the counter's
    gate): every counter forced onto them (LC_WCTR_MINW=1), against the oracle as sets with the
    per-config :last-op and the newest, and against the grid kernel's report (LC_WIDE_CONFIGS=0)."""
    monkeypatch.setenv("LC_WCTR_MINW", "1")
    found = carried = 0
    for t in range(30):
        h = synth.gen_counter(80, 4, 0.1, 9000 + t, invalid=True, n_crashed=t % 3)
        g = _lib.check(2, 0, h)
        assert int(_lib.check_stats()["wide_histories"]) == 1
        e = oracle.check_one("counter", h)
        assert int(g["valid"][0]) == e["valid"]
        if e["valid"] != 0:
            continue
        carried += _configs_vs_oracle(h, f"t={t}")
        found += 1
        if t % 5 == 0:
            a = _lib.failure_configs(0, 1 << 12, with_last=True)
            monkeypatch.setenv("LC_WIDE_CONFIGS", "0")
            b = _lib.failure_configs(0, 1 << 12, with_last=True)
            monkeypatch.delenv("LC_WIDE_CONFIGS")
            assert sorted(zip(a[0], a[2])) == sorted(zip(b[0], b[2])), t  # (configs with their :last-op)
            assert sorted(a[1]) == sorted(b[1]) and a[3] == b[3], t
    assert found > 5 and carried > 0
