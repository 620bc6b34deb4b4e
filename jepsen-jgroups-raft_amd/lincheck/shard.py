"""Multi-GPU sharding of the hot path, one process per GPU under
torch.distributed (backend "nccl" = RCCL over xGMI; "gloo" in the CPU tests).

Axis 1 (independent keys, C1/C3): `key_range` — each rank checks its own keys, no data-path
collective; the host gathers verdicts (jepsen.independent's merge-valid).
Axis 3 (counter bounds scan, C5): `bounds_shard` splits one history's entries into contiguous
blocks; each rank scans its block (plus the halo back to its earliest observation's
invocation) after ONE exchange: an all-gather of five int64 sums per rank, turned into the
exclusive prefix of the ranks before it (`exclusive_sums`). The verdict is the earliest
rejected completion over all ranks (`first_bad`, an all-reduce MIN)."""
from __future__ import annotations

import numpy as np

NONE = np.iinfo(np.int64).max


def key_range(n_keys: int, rank: int, world: int):
    """Contiguous, balanced key blocks."""
    q, r = divmod(n_keys, world)
    b = rank * q + min(rank, r)
    return b, b + q + (1 if rank < r else 0)


def bounds_shard(n_entries: int, rank: int, world: int):
    """The entries whose completions rank `rank` owns (contiguous, balanced)."""
    return key_range(n_entries, rank, world)


def _dev(tdist):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if tdist.get_backend() == "nccl" \
        else torch.device("cpu")


def exclusive_sums(sums, tdist=None):
    """All-gather every rank's five block sums; return the sums of the ranks before this one."""
    sums = np.asarray(sums, dtype=np.int64)
    if tdist is None or not tdist.is_initialized() or tdist.get_world_size() == 1:
        return np.zeros(5, np.int64)
    import torch
    dev = _dev(tdist)
    mine = torch.as_tensor(sums, device=dev)
    allv = [torch.empty_like(mine) for _ in range(tdist.get_world_size())]
    tdist.all_gather(allv, mine)
    r = tdist.get_rank()
    excl = torch.zeros(5, dtype=torch.int64, device=dev)
    for k in range(r):
        excl += allv[k]
    return excl.cpu().numpy()


def first_bad(bad_idx: int, tdist=None):
    """Earliest rejected :index over all ranks (-1 when every shard passed)."""
    v = NONE if bad_idx < 0 else int(bad_idx)
    if tdist is not None and tdist.is_initialized() and tdist.get_world_size() > 1:
        import torch
        t = torch.tensor([v], dtype=torch.int64, device=_dev(tdist))
        tdist.all_reduce(t, op=tdist.ReduceOp.MIN)
        v = int(t.item())
    return -1 if v == NONE else v
