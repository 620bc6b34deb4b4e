"""TEST INFRASTRUCTURE: a pure-Python stand-in for one rank's lc_part plan (same interface as
lincheck._lib.PartPlan), so the multi-rank level protocol of lincheck.partition.search runs
under gloo on CPUs without a GPU. It restates the per-rank semantics of csrc/part.hip (owner
by hash of the config with the returning slot cleared, DIRECT returns, S / OUT dedup sets)
over its own small encoder of the history (knossos.history pairing, :fail dropped, lowest free
slot first, cas-register memo ids; the same contract as csrc/encode.cpp)."""
from __future__ import annotations

import numpy as np

ANY, NEVER, KEEP = -1, -2, -1
DIRECT = 1 << 63
M64 = (1 << 64) - 1


def mix64(x: int) -> int:
    x &= M64
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & M64
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & M64
    x ^= x >> 33
    return x


def encode_register(h, hist=0):
    """-> (steps, mask_bits); steps = [(slot j, [(slot, a, b) invocations before it],
    :ok :index, invocation :index)]"""
    b, e = int(h.off[hist]), int(h.off[hist + 1])
    idx = lambda i: int(h.index[i]) if h.index is not None else i - b  # noqa: E731
    ops, pend, op_of = [], {}, {}
    for i in range(b, e):
        p, t = int(h.process[i]), int(h.type[i])
        if t == 0:
            op_of[i] = len(ops)
            pend[p] = len(ops)
            ops.append({"f": int(h.f[i]), "vf": int(h.vflags[i]), "v0": int(h.v0[i]),
                        "v1": int(h.v1[i]), "st": 0, "inv": i})
        else:
            k = pend.pop(p)
            op_of[i] = k
            ops[k]["st"] = t
            if t == 1:
                ops[k].update(vf=int(h.vflags[i]), v0=int(h.v0[i]), v1=int(h.v1[i]))
    sid = {}
    for o in ops:
        if o["st"] == 2:
            continue
        if o["f"] == 1 and o["vf"] == 1:
            sid.setdefault(o["v0"], len(sid) + 1)
        if o["f"] == 2 and o["vf"] == 2:
            sid.setdefault(o["v1"], len(sid) + 1)
    for o in ops:
        if o["f"] == 1:
            o["a"], o["b"] = ANY, (0 if o["vf"] == 0 else sid[o["v0"]])
        elif o["f"] == 2:
            o["a"], o["b"] = sid.get(o["v0"], NEVER), sid[o["v1"]]
        else:
            o["a"], o["b"] = (ANY if o["vf"] == 0 else sid.get(o["v0"], NEVER)), KEEP
    used, steps, invs, width = set(), [], [], 1
    for i in range(b, e):
        k = op_of[i]
        o = ops[k]
        t = int(h.type[i])
        if t == 0:
            if o["st"] == 2:
                continue
            s = 0
            while s in used:
                s += 1
            used.add(s)
            o["slot"] = s
            width = max(width, s + 1)
            invs.append((s, o["a"], o["b"]))
        elif t == 1:
            steps.append((o["slot"], invs, idx(i), idx(o["inv"])))
            invs = []
            used.discard(o["slot"])
    return steps, width


class MockPartPlan:
    H_CAPACITY = -7

    def __init__(self, h, hist=0, rank=0, world=1, set_cap=None, pack_fail_at=None):
        self.rank, self.world = rank, world
        self.set_cap = set_cap  # capacity of this rank's closure set (None: unbounded)
        self.pack_fail_at = pack_fail_at  # the pack call (0-based) that overflows (None: never)
        self.packs = self.absorbs = 0
        self.steps, self.mask_bits = encode_register(h, hist)
        self.n_steps = len(self.steps)
        self.err = 0
        self.ops = {}
        self.live = 0
        self.F = [0] if rank == 0 else []
        self.explored = 0

    def owner(self, k):
        return ((mix64(k) >> 32) * self.world) >> 32

    def step_begin(self, t, stream=None):
        j, invs, _, _ = self.steps[t]
        for s, a, b in invs:
            self.ops[s] = (a, b)
            self.live |= 1 << s
        self.bitj = 1 << j
        self.S, self.O, self.OUT = set(), set(), []
        self.L = self.F

    def expand(self, stream=None):
        mb = self.mask_bits
        mmask = (1 << mb) - 1
        self.stage = [[] for _ in range(self.world)]
        for c in self.L:
            if c & self.bitj:
                r = c & ~self.bitj
                self.stage[self.owner(r)].append(r | DIRECT)
                continue
            st = c >> mb
            for k in range(mb):
                if not (self.live >> k) & 1 or (c >> k) & 1:
                    continue
                a, b = self.ops[k]
                if a == ANY or a == st:
                    ns = st if b < 0 else b
                    c2 = (ns << mb) | (c & mmask) | (1 << k)
                    self.stage[self.owner(c2 & ~self.bitj)].append(c2)
        return np.array([len(s) for s in self.stage], np.int64)

    def pack(self, dst, stream=None):
        self.packs += 1
        if self.pack_fail_at is not None and self.packs - 1 == self.pack_fail_at:
            from lincheck._lib import CapacityError
            raise CapacityError(f"rank {self.rank}: send staging full")
        flat = [x for s in self.stage for x in s]
        # int64 view of the u64 keys (DIRECT is the sign bit)
        dst[:len(flat)] = __import__("torch").tensor(
            np.array(flat, dtype=np.uint64).view(np.int64), dtype=dst.dtype)

    def absorb(self, recv, n, stream=None):
        self.absorbs += 1
        keys = [x for s in self.stage for x in s] if recv is None else \
            [int(x) & M64 for x in recv[:n].tolist()]
        nxt = []
        for key in keys:
            if key & DIRECT:
                o = key & ~DIRECT
                if o not in self.O:
                    self.O.add(o)
                    self.OUT.append(o)
            elif key not in self.S:
                if self.set_cap is not None and len(self.S) >= self.set_cap:
                    from lincheck._lib import CapacityError
                    raise CapacityError(f"rank {self.rank}: closure set full ({self.set_cap})")
                self.S.add(key)
                self.explored += 1
                if key & self.bitj:
                    o = key & ~self.bitj
                    if o not in self.O:
                        self.O.add(o)
                        self.OUT.append(o)
                else:
                    nxt.append(key)
        self.L = nxt

    def step_end(self, stream=None):
        self.F = self.OUT
        self.live &= ~self.bitj
        return len(self.F)

    def results(self, t, stream=None):
        _, _, cmp_idx, inv_idx = self.steps[t] if 0 <= t < self.n_steps else (0, 0, -1, -1)
        prev = self.steps[t - 1][2] if 0 < t <= self.n_steps else -1
        return self.explored, cmp_idx, inv_idx, prev

    def close(self):
        pass
