"""One huge history across GPUs (SURVEY §8(e) axis 2): the frontier of a single cas-register
history is partitioned by config hash over the ranks of a torch.distributed group (one process
per GPU; backend "nccl" = RCCL over xGMI, "gloo" in the CPU tests), with ONE all-to-all of
candidate configs per BFS level.

`search` drives any plan with the lincheck._lib.PartPlan interface (the HIP plan, or the
numpy stand-in the CPU tests use) through the level protocol of include/lincheck.h:

    per RETURN step t:  step_begin(t)
      per level:        counts = expand()                 (candidates per destination rank)
                        all-gather counts                 (every rank learns the level's
                                                           global total: 0 ends the step)
                        pack(send); all-to-all; absorb(recv)
      step_end()        -> this rank's frontier part; all-reduce SUM = 0 => not linearizable

The verdict, the failing :ok completion and the explored count (sum over ranks) are the same
as knossos.linear/analysis [ext] on the whole history (register.clj:109-111) and as lc_check:
every quantity is a set cardinality, independent of the partition.
"""
from __future__ import annotations

import time

import numpy as np

from . import _lib


class _Exchange:
    """The collectives of one level, over a torch.distributed group (or none at world 1)."""

    def __init__(self, tdist, device):
        self.tdist = tdist
        self.world = tdist.get_world_size() if tdist is not None else 1
        self.rank = tdist.get_rank() if tdist is not None else 0
        self.device = device
        self.nccl = tdist is not None and tdist.get_backend() == "nccl"
        self.cdev = device if self.nccl else "cpu"  # where collective tensors live
        self.bytes = 0

    def gather_counts(self, counts: np.ndarray, over: bool):
        """All-gather every rank's per-destination counts plus its capacity flag ->
        ([src][dst] counts, whether any rank overflowed)."""
        import torch
        w = self.world + 1
        mine = torch.as_tensor(np.append(counts, int(over)), dtype=torch.int64).to(self.cdev)
        allv = torch.empty(self.world * w, dtype=torch.int64, device=self.cdev)
        self.tdist.all_gather_into_tensor(allv, mine) if self.nccl else \
            self.tdist.all_gather(list(allv.view(self.world, w).unbind(0)), mine)
        a = allv.view(self.world, w).cpu().numpy()
        return a[:, :self.world], bool(a[:, self.world].any())

    def all_to_all(self, send, n_send: int, in_splits, out_splits, recv_pool):
        """send[:n_send] (device tensor, by destination) -> received device tensor."""
        import torch
        n_recv = int(sum(out_splits))
        if self.nccl:
            recv = recv_pool(n_recv)
            self.tdist.all_to_all_single(recv[:n_recv], send[:n_send], output_split_sizes=out_splits,
                                         input_split_sizes=in_splits)
        else:
            rc = torch.empty(n_recv, dtype=torch.int64)
            self.tdist.all_to_all_single(rc, send[:n_send].cpu(), output_split_sizes=out_splits,
                                         input_split_sizes=in_splits)
            recv = rc.to(self.device, non_blocking=False) if self.device != "cpu" else rc
        self.bytes += 8 * (n_send + n_recv)
        return recv, n_recv

    def sum(self, v: int, over: bool = False):
        """All-reduce SUM of v and of the capacity flags -> (sum, whether any rank overflowed)."""
        import torch
        t = torch.tensor([int(v), int(over)], dtype=torch.int64, device=self.cdev)
        self.tdist.all_reduce(t)
        return int(t[0].item()), bool(t[1].item())


def search(plan, tdist=None, device="cpu", stream=None, max_steps=None, device_loop=True):
    """Run the partitioned search of `plan` (this rank's part) to the end. Returns
    {"valid": 1/0/2, "fail_step", "fail_idx", "fail_inv", "prev_ok", "explored", "err",
     "steps", "levels", "exchanged_bytes", "wall_s"} — identical on every rank. At world 1 a
    plan with `run` (the HIP plan) keeps the whole level loop on the device (lc_part_run)
    unless device_loop is False."""
    ex = _Exchange(tdist, device)
    if ex.world == 1 and device_loop and hasattr(plan, "run") and not plan.err:
        return _search_device(plan, stream, max_steps)
    world, rank = ex.world, ex.rank
    state = {"send": None, "recv": None}

    def buf(name, n):
        import torch
        b = state[name]
        if b is None or b.numel() < n:
            b = torch.empty(max(n, 1 << 16) * 2, dtype=torch.int64, device=device)
            state[name] = b
        return b

    t0 = time.perf_counter()
    n_steps = plan.n_steps if max_steps is None else min(plan.n_steps, max_steps)
    levels = 0
    fail_t = -1
    valid, err = 1, 0
    if plan.err:
        return {"valid": 2, "fail_step": -1, "fail_idx": -1, "fail_inv": -1, "prev_ok": -1,
                "explored": 0, "err": plan.err, "steps": 0, "levels": 0, "exchanged_bytes": 0,
                "wall_s": 0.0}
    # Capacity is per rank (this rank's hash sets and lists). A rank that overflows stops
    # calling its plan but keeps taking part in the level's collectives with empty sends; its
    # flag rides on the next count all-gather or frontier all-reduce, so every rank leaves at
    # the same collective and reports :unknown together (no mismatched collectives).
    over = False

    def attempt(fn, *a):
        nonlocal over
        if over:
            return None
        try:
            return fn(*a)
        except _lib.CapacityError:
            over = True
            return None

    t = -1
    any_over = False
    for t in range(n_steps):
        attempt(plan.step_begin, t, stream)
        while True:
            counts = attempt(plan.expand, stream)
            if counts is None:
                counts = np.zeros(world, np.int64)
            levels += 1
            if world == 1:
                any_over = over
                n = int(counts[0])
                if n == 0 or over:
                    break
                attempt(plan.absorb, None, n, stream)
                continue
            # pack before the count exchange: a rank whose pack overflows then announces zero
            # counts with its flag, so no peer ever absorbs a stale send buffer
            n_send = int(counts.sum())
            send = buf("send", n_send) if n_send else None
            if n_send:
                attempt(plan.pack, send, stream)
            if over:
                counts, n_send = np.zeros(world, np.int64), 0
            cm, any_over = ex.gather_counts(counts, over)
            if any_over or int(cm.sum()) == 0:
                break
            if send is None:
                send = buf("send", 1)
            recv, n_recv = ex.all_to_all(send, n_send, counts.tolist(), cm[:, rank].tolist(),
                                         lambda n: buf("recv", n))
            attempt(plan.absorb, recv, n_recv, stream)
        if any_over:
            break
        mine = attempt(plan.step_end, stream)
        mine = 0 if mine is None else mine
        total, any_over = (mine, over) if world == 1 else ex.sum(mine, over)
        if any_over:
            break
        if total == 0:
            fail_t = t
            valid = 0
            break
    if any_over:
        valid, err = 2, _lib.PartPlan.H_CAPACITY
    res = attempt(plan.results, fail_t if fail_t >= 0 else t, stream) or (0, -1, -1, -1)
    expl, fidx, finv, prev = res
    explored = expl if world == 1 else ex.sum(expl)[0]
    st = plan.stats() if hasattr(plan, "stats") else {"kernel_ms": 0.0, "alg_bytes": 0.0}
    return {"valid": valid, "fail_step": fail_t,
            "fail_idx": fidx if valid == 0 else -1, "fail_inv": finv if valid == 0 else -1,
            "prev_ok": prev if valid == 0 else -1, "explored": explored, "err": err,
            "steps": t + 1, "levels": levels, "exchanged_bytes": ex.bytes,
            "kernel_ms": st["kernel_ms"], "alg_bytes": st["alg_bytes"],
            "wall_s": time.perf_counter() - t0}


def _search_device(plan, stream, max_steps):
    t0 = time.perf_counter()
    try:
        steps, fail_t, levels, explored = plan.run(stream, -1 if max_steps is None else max_steps)
        valid, err = (0 if fail_t >= 0 else 1), 0
    except _lib.CapacityError:
        steps, fail_t, levels, explored = 0, -1, 0, 0
        valid, err = 2, _lib.PartPlan.H_CAPACITY
    res = plan.results(fail_t if fail_t >= 0 else steps - 1, stream)
    if valid == 2:
        explored = res[0]
    st = plan.stats()
    return {"valid": valid, "fail_step": fail_t,
            "fail_idx": res[1] if valid == 0 else -1, "fail_inv": res[2] if valid == 0 else -1,
            "prev_ok": res[3] if valid == 0 else -1, "explored": explored, "err": err,
            "steps": steps, "levels": levels, "exchanged_bytes": 0,
            "kernel_ms": st["kernel_ms"], "alg_bytes": st["alg_bytes"],
            "wall_s": time.perf_counter() - t0}


def check_partitioned(h, hist: int = 0, tdist=None, device_index: int | None = None,
                      capacity_log2: int = 0, device_loop: bool = True):
    """Check history `hist` of h with its frontier partitioned over the ranks of `tdist`
    (torch.distributed, initialised; None = one rank) on this rank's GPU."""
    world = tdist.get_world_size() if tdist is not None else 1
    rank = tdist.get_rank() if tdist is not None else 0
    stream = None
    device = "cpu"
    if device_index is None:
        device_index = 0
    if world > 1:
        import torch
        device = torch.device("cuda", device_index)
        torch.cuda.set_device(device)
        stream = torch.cuda.current_stream(device).cuda_stream
    plan = _lib.PartPlan(h, hist=hist, rank=rank, world=world, device=device_index,
                         capacity_log2=capacity_log2)
    try:
        return search(plan, tdist, device, stream, device_loop=device_loop)
    finally:
        plan.close()
