"""CPU tests of bench.py's host-side pieces (no GPU): the cpu_baseline leg (the whole workload,
the fastest of several passes, the per-key figures beside it) and the whole-history fixtures
the single-history lines quote."""
import importlib.util
import os

import pytest

from lincheck import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_cpu_baseline_whole_workload_fastest_pass(bench):
    h = synth.gen_config("c1")
    cpu, res, sample, hs = bench.cpu_baseline(h, "cas-register", 1.0, 2, full=True, reps=2)
    assert sample == list(range(h.n_hist)) and len(res) == h.n_hist
    assert len(cpu["pass_walls_s"]) == 2
    assert cpu["wall_s"] == pytest.approx(min(cpu["pass_walls_s"]), abs=1e-3)
    w = cpu["wall_s"]  # (rounded to 1 ms)
    assert hs.n_ops() / (w + 6e-4) <= cpu["value"] <= hs.n_ops() / max(w - 6e-4, 1e-9)
    assert "fastest of 2 passes" in cpu["sample"] and cpu["cores"] == 2
    pk = cpu["per_key"]
    assert pk["max_s"] <= pk["sum_s"] and pk["wall_bound_s"] == pytest.approx(max(pk["sum_s"] / 2, pk["max_s"]),
                                                                                abs=1e-3)


def test_cpu_baseline_quick_sample_is_one_pass(bench):
    h = synth.gen_config("c3", scale=0.1)
    cpu, res, sample, hs = bench.cpu_baseline(h, "cas-register", 1.0, 2, full=False, reps=1)
    assert len(cpu["pass_walls_s"]) == 1 and "a quick sample" in cpu["sample"]
    assert sample == list(range(0, h.n_hist, max(1, h.n_hist // 50)))


@pytest.mark.parametrize("workload", ["c4", "c2c", "c2c4", "c5x"])
def test_golden_fixture_for_single_history_lines(bench, workload):
    fx = bench.golden_fixture(workload)
    assert fx is not None and fx["explored"] > 0 and fx["provenance"]["wall_s"] > 0
    assert bench.golden_fixture("c3") is None


def _run_bench(argv, env_extra, timeout=240):
    import subprocess
    import sys
    env = dict(os.environ, **env_extra)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if k not in env_extra:
            env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + argv, capture_output=True,
                          text=True, timeout=timeout, env=env, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    """plain `python3 bench.py --gpus N` (the driver's scaling command) starts
    N ranks itself under torch.distributed.run and relays rank 0's one JSON line. The GPU work is
    skipped by the LC_BENCH_PROTOCOL_ONLY hook so the launcher runs here (gloo, no GPU)."""
    import json
    r = _run_bench(["--gpus", str(n), "--steps", "2", "--warmup", "1"], {"LC_BENCH_PROTOCOL_ONLY": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_seen"] == n and out["steps"] == 2


def test_bench_refuses_gpus_world_mismatch():
    """Under an external launcher, --gpus must equal WORLD_SIZE (no silent one-rank runs)."""
    r = _run_bench(["--gpus", "8", "--steps", "1", "--warmup", "0"],
                   {"WORLD_SIZE": "1", "RANK": "0", "LC_BENCH_PROTOCOL_ONLY": "1"}, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
