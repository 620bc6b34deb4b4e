"""History encoding: Jepsen op maps -> the SoA int arrays the C-ABI takes.

Mirrors the op shapes the reference's clients produce:
  * register: read invoke value nil, ok value long-or-nil (register.clj:16-19, :74-75);
    write keeps its value (:77-78); cas ok -> [old new] (:83); cas failure -> :fail (:84)
  * counter: read ok -> long (counter.clj:82-83);
    add/decr keep the delta; *-and-get ok -> [delta result] (:91-93)
  * independent keys: value = (tuple k v) (jepsen.independent [ext]; register.clj:75, :83)
  * error classification (client.clj:52-63): timeouts of non-idempotent ops -> :info

Encoding (include/lincheck.h): type 0 invoke / 1 ok / 2 fail / 3 info;
f 0 read / 1 write / 2 cas / 3 add / 4 decr / 5 add-and-get / 6 decr-and-get / 7 inspect;
vflags 0 nil / 1 scalar (v0) / 2 pair (v0, v1).
  * election (leader.clj:14-17, :38-40): :inspect invokes with [nil 0], completes with
    [leader term ...]; encoded as the pair (leader id, term), the id interned per process from
    serialize-leader's name (nil and "null" -> -1, leader.clj:51-54)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, Iterable, List, NamedTuple, Optional, Sequence

import numpy as np

TYPE_CODES = {"invoke": 0, "ok": 1, "fail": 2, "info": 3}
TYPE_NAMES = {v: k for k, v in TYPE_CODES.items()}
F_CODES = {"read": 0, "write": 1, "cas": 2, "add": 3, "decr": 4,
           "add-and-get": 5, "decr-and-get": 6, "inspect": 7}
F_NAMES = {v: k for k, v in F_CODES.items()}
V_NIL, V_SCALAR, V_PAIR = 0, 1, 2


class KV(NamedTuple):
    """jepsen.independent/tuple: a [key value] pair carried in an op's :value."""
    key: Any
    value: Any


def tuple_(k, v) -> KV:
    return KV(k, v)


def _kw(x) -> str:
    s = str(x)
    return s[1:] if s.startswith(":") else s


F_INSPECT = F_CODES["inspect"]
_LEADER_IDS: Dict[str, int] = {"null": -1}
_LEADER_NAMES: Dict[int, Optional[str]] = {-1: None}


def leader_id(addr) -> int:
    """The id of serialize-leader(addr) (leader.clj:51-54): equal names, equal ids."""
    name = "null" if addr is None else str(addr)
    i = _LEADER_IDS.get(name)
    if i is None:
        i = _LEADER_IDS[name] = len(_LEADER_IDS) - 1
        _LEADER_NAMES[i] = name
    return i


def _encode_inspect(v):
    """[leader term ...] -> (V_PAIR, leader id, term); nil stays nil ((leader nil, term nil))."""
    if v is None:
        return V_NIL, 0, 0
    if not isinstance(v, (list, tuple)) or len(v) < 2 or v[1] is None:
        raise ValueError(f":inspect value must be [leader term ...], got {v!r}")
    return V_PAIR, leader_id(v[0]), int(v[1])


def _encode_value(v):
    if v is None:
        return V_NIL, 0, 0
    if isinstance(v, (list, tuple)) and not isinstance(v, KV):
        if len(v) != 2:
            raise ValueError(f"pair value must have 2 elements, got {v!r}")
        a, b = v
        if a is None or b is None:
            raise ValueError(f"nil inside a pair value is not supported: {v!r}")
        return V_PAIR, int(a), int(b)
    return V_SCALAR, int(v), 0


@dataclass
class History:
    """One or many histories, concatenated; `off` has n_hist+1 entries."""
    off: np.ndarray       # int64 [n_hist+1]
    index: np.ndarray     # int64 [n]  (the ops' :index)
    process: np.ndarray   # int32 [n]
    type: np.ndarray      # int8  [n]
    f: np.ndarray         # int8  [n]
    v0: np.ndarray        # int64 [n]
    v1: np.ndarray        # int64 [n]
    vflags: np.ndarray    # int8  [n]
    keys: Optional[list] = None  # per sub-history key (independent), else None

    @property
    def n_hist(self) -> int:
        return len(self.off) - 1

    @property
    def n(self) -> int:
        return int(self.off[-1])

    def n_ops(self) -> int:
        """Client operations = invocations (counted before :fail removal)."""
        return int(np.count_nonzero(self.type == 0))

    def sub(self, h: int) -> "History":
        b, e = int(self.off[h]), int(self.off[h + 1])
        return History(np.array([0, e - b], np.int64), self.index[b:e], self.process[b:e],
                       self.type[b:e], self.f[b:e], self.v0[b:e], self.v1[b:e],
                       self.vflags[b:e], None if self.keys is None else [self.keys[h]])

    def select(self, hs: Sequence[int]) -> "History":
        return concat([self.sub(int(h)) for h in hs])

    def to_ops(self, h: int = 0) -> List[Dict[str, Any]]:
        b, e = int(self.off[h]), int(self.off[h + 1])
        out = []
        for i in range(b, e):
            vf = int(self.vflags[i])
            v = None if vf == V_NIL else (int(self.v0[i]) if vf == V_SCALAR
                                          else [int(self.v0[i]), int(self.v1[i])])
            if int(self.f[i]) == F_INSPECT and vf == V_PAIR:
                v = [_LEADER_NAMES.get(int(self.v0[i])), int(self.v1[i])]
            out.append({"process": int(self.process[i]), "index": int(self.index[i]),
                        "type": TYPE_NAMES[int(self.type[i])], "f": F_NAMES[int(self.f[i])],
                        "value": v})
        return out

    def arrays(self):
        return (self.off, self.index, self.process, self.type, self.f, self.v0, self.v1,
                self.vflags)


def from_columns(index, process, type_, f, v0, v1, vflags, off=None, keys=None) -> History:
    n = len(type_)
    if off is None:
        off = [0, n]
    return History(np.ascontiguousarray(off, np.int64), np.ascontiguousarray(index, np.int64),
                   np.ascontiguousarray(process, np.int32), np.ascontiguousarray(type_, np.int8),
                   np.ascontiguousarray(f, np.int8), np.ascontiguousarray(v0, np.int64),
                   np.ascontiguousarray(v1, np.int64), np.ascontiguousarray(vflags, np.int8),
                   keys)


def client_op(op: Dict[str, Any]) -> bool:
    """Only client ops (integer :process) reach the model (nemesis ops are excluded)."""
    p = op.get("process")
    return isinstance(p, (int, np.integer)) and not isinstance(p, bool)


def encode(ops: Iterable[Dict[str, Any]], unwrap_key: bool = False) -> History:
    """Encode one history (a sequence of op dicts) into SoA arrays."""
    idx, proc, typ, fs, a0, a1, vfl = [], [], [], [], [], [], []
    for pos, op in enumerate(ops):
        if not client_op(op):
            continue
        v = op.get("value")
        if unwrap_key and isinstance(v, KV):
            v = v.value
        f = F_CODES[_kw(op["f"])]
        vf, x, y = _encode_inspect(v) if f == F_INSPECT else _encode_value(v)
        idx.append(int(op.get("index", pos)))
        proc.append(int(op["process"]))
        typ.append(TYPE_CODES[_kw(op["type"])])
        fs.append(f)
        a0.append(x)
        a1.append(y)
        vfl.append(vf)
    return from_columns(idx, proc, typ, fs, a0, a1, vfl)


def subhistories(ops: Iterable[Dict[str, Any]]) -> History:
    """jepsen.independent/subhistory [ext]: group ops with (tuple k v) values by key, keep
    order, unwrap values. Ops whose value is not a tuple (e.g. nemesis ops) are dropped.
    Keys come out in first-appearance order."""
    groups: Dict[Any, list] = {}
    for pos, op in enumerate(ops):
        v = op.get("value")
        if not isinstance(v, KV) or not client_op(op):
            continue
        o = dict(op)
        o.setdefault("index", pos)
        groups.setdefault(v.key, []).append(o)
    hs = [encode(g, unwrap_key=True) for g in groups.values()]
    h = concat(hs) if hs else from_columns([], [], [], [], [], [], [])
    h.keys = list(groups.keys())
    return h


def concat(hs: Sequence[History]) -> History:
    if not hs:
        return from_columns([], [], [], [], [], [], [], off=[0])
    # every input keeps its own sub-histories
    offs, base = [np.zeros(1, np.int64)], 0
    for h in hs:
        offs.append(np.asarray(h.off[1:], np.int64) - int(h.off[0]) + base)
        base += h.n
    off = np.concatenate(offs)
    keys = None
    if all(h.keys is not None for h in hs):
        keys = [k for h in hs for k in h.keys]
    return History(off, *(np.concatenate([getattr(h, a) for h in hs])
                          for a in ("index", "process", "type", "f", "v0", "v1", "vflags")),
                   keys=keys)
