"""GPU parity against the oracle-pinned wide and full-size INVALID fixtures.

tests/golden/pin_wide.py ran the CPU oracle once per history in the build container and wrote
tests/golden/wide_<name>_oracle.json: the crash ramp's real wide frontiers (K = 13 and 14,
live width 27, and K = 16, width 30, where its frontier fitted memory) on the HBM tables
(csrc/wide.hip), the K = 13 history perturbed at 50 % (the pipelined HBM-table kernel stops
mid-history with later steps in flight), C4 perturbed at 15 % (the rotated 128-tile team stops
mid-history), and the 1M-op counter c5x perturbed at 2 % (the counter closure tables stop
mid-history). Each test regenerates the history, checks its digest, runs it through the C-ABI
and compares verdict, the failing :index triple (raft_test.clj:29-65's invalid shape) and the
explored count with the fixture, and checks which kernel decided it."""
import json
import os
import sys

import pytest

from lincheck import _lib

pytestmark = pytest.mark.gpu
GOLD_DIR = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLD_DIR)
import pin_wide  # noqa: E402

# the kernel each fixture must take (lc_check_stats counters)
PATH = {"ramp11s": "wide_histories", "ramp10c17": "wide_histories", "ramp11c17": "wide_histories",
        "ramp13": "wide_histories", "ramp14": "wide_histories", "ramp16": "wide_histories",
        "ramp13x50": "wide_histories", "c4x15": "dense_histories", "c4x15n": "dense_histories", "c5xx2": "ctab_histories"}
PINNED = [n for n in pin_wide.GEN if os.path.exists(pin_wide.path_of(n))]


@pytest.fixture(scope="module", autouse=True)
def _device():
    if _lib.load().lc_device_count() < 1:
        pytest.fail("no HIP device on a GPU run: the checker has no CPU fallback")


@pytest.mark.parametrize("name", PINNED)
def test_gpu_matches_pinned_fixture(name):
    fx = json.load(open(pin_wide.path_of(name)))
    model, _, gen = pin_wide.GEN[name]
    h = gen()
    assert (h.n, pin_wide.digest(h)) == (fx["n_entries"], fx["digest"])
    g = _lib.check(_lib.MODEL_KIND[model], 0, h)
    st = _lib.check_stats()
    assert int(st[PATH[name]]) == 1, (name, PATH[name], st)
    if PATH[name] != "wide_histories":
        assert int(st["wide_histories"]) == 0, (name, st)
    got = (int(g["valid"][0]), int(g["fail_idx"][0]), int(g["fail_inv"][0]), int(g["prev_ok"][0]),
           int(g["explored"][0]))
    exp = (fx["valid"], fx["fail_idx"], fx["fail_inv_idx"], fx["prev_ok_idx"], fx["explored"])
    assert got == exp, (name, got, exp)
