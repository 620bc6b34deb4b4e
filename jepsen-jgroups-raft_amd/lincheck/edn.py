"""A small EDN reader for stored Jepsen histories (`store/<test>/<time>/history.edn`, the
directory the reference's .gitignore:16 keeps out of git; written by jepsen.store [ext] at the
end of every `lein run test`, raft.clj:100). Enough of EDN for op maps: nil / booleans /
integers / floats / strings / characters, keywords and symbols, vectors, lists, maps, sets,
comments, `#_` discard, and tagged literals. A tagged map is read as the map itself, so
`#jepsen.history.Op{...}` is an op. `#jepsen.independent.Tuple{:key k :value v}` becomes a
lincheck.history.KV, as do the two-element vectors jepsen.independent tuples print as.

Keywords come back as plain strings without the colon (":invoke" -> "invoke"), so the ops
read here feed lincheck.history.encode / subhistories unchanged.
"""
from __future__ import annotations

import re
from typing import Any, Dict, Iterator, List

from .history import KV

_WS = set(" \t\r\n,")
_DELIM = set("()[]{}\"; \t\r\n,")
_INT = re.compile(r"^[+-]?\d+N?$")
_FLOAT = re.compile(r"^[+-]?\d+(\.\d*)?([eE][+-]?\d+)?M?$")
_CHARS = {"newline": "\n", "space": " ", "tab": "\t", "return": "\r", "backspace": "\b",
          "formfeed": "\f"}


class Keyword(str):
    """An EDN keyword (compares equal to its name without the colon)."""


class Tagged:
    def __init__(self, tag: str, value: Any):
        self.tag, self.value = tag, value

    def __repr__(self):
        return f"#{self.tag} {self.value!r}"


class EdnError(ValueError):
    pass


class _Reader:
    def __init__(self, text: str):
        self.s = text
        self.i = 0

    def _skip(self):
        s, n = self.s, len(self.s)
        while self.i < n:
            c = s[self.i]
            if c in _WS:
                self.i += 1
            elif c == ";":
                j = s.find("\n", self.i)
                self.i = n if j < 0 else j + 1
            else:
                break

    def at_end(self) -> bool:
        self._skip()
        return self.i >= len(self.s)

    def read(self) -> Any:
        self._skip()
        if self.i >= len(self.s):
            raise EdnError("unexpected end of input")
        c = self.s[self.i]
        if c == "(":
            self.i += 1
            return self._seq(")")
        if c == "[":
            self.i += 1
            return self._seq("]")
        if c == "{":
            self.i += 1
            items = self._seq("}")
            if len(items) % 2:
                raise EdnError("map with an odd number of forms")
            return {_hashable(items[k]): items[k + 1] for k in range(0, len(items), 2)}
        if c == '"':
            return self._string()
        if c == "\\":
            return self._char()
        if c == "#":
            return self._dispatch()
        if c in ")]}":
            raise EdnError(f"unbalanced {c!r} at {self.i}")
        return self._atom()

    def _seq(self, close: str) -> List[Any]:
        out = []
        while True:
            self._skip()
            if self.i >= len(self.s):
                raise EdnError(f"missing {close!r}")
            if self.s[self.i] == close:
                self.i += 1
                return out
            v = self.read()
            if v is not _DISCARD:
                out.append(v)

    def _string(self) -> str:
        self.i += 1
        out = []
        s = self.s
        while True:
            if self.i >= len(s):
                raise EdnError("unterminated string")
            c = s[self.i]
            if c == '"':
                self.i += 1
                return "".join(out)
            if c == "\\":
                e = s[self.i + 1]
                self.i += 2
                if e == "u":
                    out.append(chr(int(s[self.i:self.i + 4], 16)))
                    self.i += 4
                else:
                    out.append({"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\"}.get(e, e))
            else:
                out.append(c)
                self.i += 1

    def _char(self) -> str:
        self.i += 1
        j = self.i + 1
        while j < len(self.s) and self.s[j] not in _DELIM:
            j += 1
        tok = self.s[self.i:j]
        self.i = j
        return _CHARS.get(tok, tok)

    def _dispatch(self) -> Any:
        s = self.s
        nxt = s[self.i + 1] if self.i + 1 < len(s) else ""
        if nxt == "{":
            self.i += 2
            return frozenset(_hashable(x) for x in self._seq("}"))
        if nxt == "_":
            self.i += 2
            self.read()
            return _DISCARD
        self.i += 1
        j = self.i
        while j < len(s) and s[j] not in _DELIM:
            j += 1
        tag = s[self.i:j]
        self.i = j
        v = self.read()
        if tag == "jepsen.independent.Tuple" and isinstance(v, dict):
            return KV(v.get("key"), v.get("value"))
        if isinstance(v, dict):  # records (#jepsen.history.Op{...}): the map itself
            return v
        return Tagged(tag, v)

    def _atom(self) -> Any:
        s = self.s
        j = self.i
        while j < len(s) and s[j] not in _DELIM:
            j += 1
        tok = s[self.i:j]
        self.i = j
        if tok == "nil":
            return None
        if tok == "true":
            return True
        if tok == "false":
            return False
        if tok.startswith(":"):
            return Keyword(tok[1:])
        if _INT.match(tok):
            return int(tok.rstrip("N"))
        if _FLOAT.match(tok):
            return float(tok.rstrip("M"))
        return tok  # symbol


_DISCARD = object()


def _hashable(x):
    if isinstance(x, list):
        return tuple(_hashable(v) for v in x)
    if isinstance(x, dict):
        return tuple(sorted((k, _hashable(v)) for k, v in x.items()))
    return x


def loads_all(text: str) -> Iterator[Any]:
    """Every top-level form of `text`."""
    r = _Reader(text)
    while not r.at_end():
        v = r.read()
        if v is not _DISCARD:
            yield v


def _op(m: Dict[Any, Any], independent: bool) -> Dict[str, Any]:
    op = {str(k): v for k, v in m.items()}
    v = op.get("value")
    # jepsen.independent tuples print as [k v] vectors (or as Tuple records, handled above)
    if independent and isinstance(v, list) and len(v) == 2 and not isinstance(v, KV):
        op["value"] = KV(v[0], v[1])
    return op


def read_history(path_or_text: str, independent: bool = False) -> List[Dict[str, Any]]:
    """Ops of a stored history: a file of one op map per line, or one vector of op maps.
    `independent`: values are [key value] tuples (the register workloads, register.clj:106)."""
    text = path_or_text
    if "\n" not in path_or_text and not path_or_text.lstrip().startswith(("{", "[", "#")):
        with open(path_or_text, encoding="utf-8") as fh:
            text = fh.read()
    forms = list(loads_all(text))
    if len(forms) == 1 and isinstance(forms[0], list):
        forms = forms[0]
    return [_op(m, independent) for m in forms if isinstance(m, dict)]
