"""Multi-rank paths on the CPU (torch.distributed gloo, world sizes 2 and 3, 127.0.0.1): the
counter bounds scan's exclusive-prefix exchange and verdict reduction (SURVEY §8(e) axis 3)
and the key/entry sharding the bench uses. The device half of a shard runs in test_gpu.py."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as tdist
import torch.multiprocessing as mp

from lincheck import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, sums_all, bads, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        excl = shard.exclusive_sums(sums_all[rank], tdist)
        fb = shard.first_bad(bads[rank], tdist)
        q.put((rank, excl.tolist(), fb))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exclusive_sums_and_first_bad_gloo(world):
    rng = np.random.default_rng(world)
    sums_all = [rng.integers(-1000, 1000, 5).astype(np.int64) for _ in range(world)]
    bads = [-1] * world
    bads[world - 1] = 77
    if world > 2:
        bads[1] = 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sums_all, bads, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (e, fb)) for r, e, fb in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        exp = np.sum(sums_all[:r], axis=0) if r else np.zeros(5, np.int64)
        assert got[r][0] == exp.tolist()
        assert got[r][1] == (12 if world > 2 else 77)


def test_exchange_identity_without_process_group():
    assert shard.exclusive_sums([1, 2, 3, 4, 5]).tolist() == [0] * 5
    assert shard.first_bad(-1) == -1 and shard.first_bad(9) == 9


@pytest.mark.parametrize("n,world", [(0, 1), (5, 3), (10, 4), (2_000_000, 8), (7, 8)])
def test_shards_partition(n, world):
    spans = [shard.bounds_shard(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
        assert e0 == b1 and b0 <= e0
    sizes = [e - b for b, e in spans]
    assert max(sizes) - min(sizes) <= 1


# ---- axis 2: one history, frontier partitioned over ranks (lincheck.partition) ----------
# The level protocol (count all-gather, all-to-all of candidates, frontier all-reduce) runs
# under gloo with a numpy stand-in for the per-rank HIP plan (tests/part_mock.py); the HIP
# plan itself runs the same driver in test_gpu.py.

def _part_histories():
    from lincheck import synth
    hs = [synth.gen_register_keys(1, 120, 5, 0.02, config_id=7, key0=k) for k in range(3)]
    hs += [synth.gen_register_keys(1, 120, 5, 0.02, config_id=7, key0=k, invalid_keys=(k,))
           for k in (7, 17)]
    return hs


def _part_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lincheck import partition
        from part_mock import MockPartPlan
        out = []
        for h in _part_histories():
            r = partition.search(MockPartPlan(h, rank=rank, world=world), tdist, "cpu", None)
            out.append((r["valid"], r["fail_idx"], r["fail_inv"], r["prev_ok"], r["explored"]))
        q.put((rank, out))
    finally:
        tdist.destroy_process_group()


def _oracle_rows():
    import oracle
    rows = []
    for h in _part_histories():
        e = oracle.check_one("cas-register", h)
        rows.append((e["valid"], e["fail_idx"] if e["valid"] == 0 else -1,
                     e["fail_inv_idx"] if e["valid"] == 0 else -1,
                     e["prev_ok_idx"] if e["valid"] == 0 else -1, e["explored"]))
    return rows


def test_partitioned_search_world1_matches_oracle():
    from lincheck import partition
    from part_mock import MockPartPlan
    exp = _oracle_rows()
    assert any(r[0] == 0 for r in exp) and any(r[0] == 1 for r in exp)
    for h, e in zip(_part_histories(), exp):
        r = partition.search(MockPartPlan(h), None, "cpu", None)
        assert (r["valid"], r["fail_idx"], r["fail_inv"], r["prev_ok"], r["explored"]) == e


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_search_gloo_matches_oracle(world):
    exp = _oracle_rows()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_part_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert [tuple(x) for x in got[r]] == exp, (r, got[r], exp)


def _overflow_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lincheck import partition
        from part_mock import MockPartPlan
        out = []
        for h in _part_histories()[:2]:
            # only rank 1's sets are small: it overflows while rank 0 is mid-protocol
            plan = MockPartPlan(h, rank=rank, world=world, set_cap=3 if rank == 1 else None)
            r = partition.search(plan, tdist, "cpu", None)
            out.append((r["valid"], r["err"]))
        # the group is still usable afterwards (no collective was left unmatched)
        t = __import__("torch").ones(1)
        tdist.all_reduce(t)
        out.append(float(t.item()))
        q.put((rank, out))
    finally:
        tdist.destroy_process_group()


def test_partitioned_overflow_on_one_rank_is_collective():
    """a rank whose closure set overflows must not leave the others waiting in a
    collective: every rank reports :unknown (LC_H_CAPACITY) at the same level."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overflow_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r][:2] == [(2, -7), (2, -7)], (r, got[r])
        assert got[r][2] == float(world)


def _pack_overflow_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lincheck import partition
        from part_mock import MockPartPlan
        h = _part_histories()[0]
        # only rank 1 overflows, in its 3rd pack: after it has expanded that level
        plan = MockPartPlan(h, rank=rank, world=world, pack_fail_at=2 if rank == 1 else None)
        r = partition.search(plan, tdist, "cpu", None)
        q.put((rank, (r["valid"], r["err"], plan.absorbs)))
    finally:
        tdist.destroy_process_group()


def test_partitioned_pack_overflow_sends_nothing_stale():
    """a rank whose pack overflows announces zero counts with its flag in the same
    count exchange, so no rank runs that level's all-to-all or absorbs a stale send buffer:
    both ranks stop after the same number of absorbs, with :unknown (LC_H_CAPACITY)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pack_overflow_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][:2] == (2, -7) and got[1][:2] == (2, -7), got
    assert got[0][2] == got[1][2] > 0, got
