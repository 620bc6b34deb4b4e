"""Writes tests/golden/kats.json — the known-answer histories for the checker.

Provenance (the reference's Clojure tests cannot run here: no JVM):
  * counter_valid / counter_invalid / counter_invalid_2 are the three histories of the
    reference's only unit tests, transcribed as data from
    test/jepsen/jgroups/raft_test.clj:6-27, :29-42, :44-65 (expected :valid? true/false/false
    — asserted there). fail_idx / prev_ok / explored come from the hand traces in
    SURVEY.md Appendix A under the §8(a) explored contract (not asserted by the reference).
  * reg_* are the hand-derived cas-register KATs of SURVEY.md Appendix A (R1-R9) plus
    edge cases; verdicts re-derived by hand (parity vs Knossos UNPINNED) and cross-checked by
    tests/brute.py in tests/test_oracle.py.
Run: python tests/golden/make_kats.py
"""
import json
import os


def op(p, i, t, f, v=None):
    return {"process": p, "index": i, "type": t, "f": f, "value": v}


def hist(*rows):
    return [op(p, i, t, f, v) for i, (p, t, f, v) in enumerate(rows)]


KATS = []


def kat(name, model, history, valid, fail_idx=-1, prev_ok=-1, explored=None, source=""):
    KATS.append({"name": name, "model": model, "history": history, "valid": valid,
                 "fail_idx": fail_idx, "prev_ok_idx": prev_ok, "explored": explored,
                 "source": source})


# ---- reference golden vectors: test/jepsen/jgroups/raft_test.clj
kat("counter_valid", "counter", [
    op(0, 0, "invoke", "add", 1), op(1, 1, "invoke", "read", None), op(1, 2, "ok", "read", 1),
    op(0, 3, "ok", "add", 1), op(1, 4, "invoke", "add-and-get", 1),
    op(1, 5, "info", "add-and-get", 1), op(0, 6, "invoke", "read", None),
    op(0, 7, "ok", "read", 1), op(2, 8, "invoke", "add-and-get", 1),
    op(2, 9, "ok", "add-and-get", [1, 2])],
    True, explored=6, source="raft_test.clj:6-27")
kat("counter_invalid", "counter", [
    op(0, 0, "invoke", "add", 1), op(0, 1, "ok", "add", 1), op(0, 2, "invoke", "read", None),
    op(0, 3, "ok", "read", 1), op(1, 4, "invoke", "read", None), op(1, 5, "ok", "read", 0)],
    False, fail_idx=5, prev_ok=3, explored=2, source="raft_test.clj:29-42")
kat("counter_invalid_2", "counter", [
    op(0, 0, "invoke", "add", 1), op(1, 1, "invoke", "read", None), op(1, 2, "ok", "read", 1),
    op(0, 3, "ok", "add", 1), op(1, 4, "invoke", "add-and-get", 1),
    op(1, 5, "info", "add-and-get", 1), op(0, 6, "invoke", "read", None),
    op(0, 7, "ok", "read", 2), op(2, 8, "invoke", "add-and-get", 1),
    op(2, 9, "ok", "add-and-get", [1, 2])],
    False, fail_idx=9, prev_ok=7, explored=4, source="raft_test.clj:44-65")

# ---- hand-derived cas-register KATs
S = "SURVEY.md Appendix A (hand-derived; Knossos parity unpinned)"
kat("reg_R1", "cas-register", hist((0, "invoke", "write", 1), (0, "ok", "write", 1),
                                   (0, "invoke", "read", None), (0, "ok", "read", 1)),
    True, explored=2, source=S)
kat("reg_R2", "cas-register", hist((0, "invoke", "write", 1), (0, "ok", "write", 1),
                                   (1, "invoke", "read", None), (1, "ok", "read", 2)),
    False, fail_idx=3, prev_ok=1, explored=1, source=S)
kat("reg_R3", "cas-register", hist((0, "invoke", "cas", [0, 1]), (0, "ok", "cas", [0, 1])),
    False, fail_idx=1, explored=0, source=S)
kat("reg_R4", "cas-register", hist((0, "invoke", "write", 1), (1, "invoke", "read", None),
                                   (1, "ok", "read", None), (0, "ok", "write", 1)),
    True, explored=4, source=S)
kat("reg_R5", "cas-register", hist((0, "invoke", "write", 3), (0, "info", "write", 3),
                                   (1, "invoke", "read", None), (1, "ok", "read", 3)),
    True, explored=2, source=S)
kat("reg_R6", "cas-register", hist((0, "invoke", "write", 3), (0, "info", "write", 3),
                                   (1, "invoke", "read", None), (1, "ok", "read", 0)),
    False, fail_idx=3, explored=1, source=S)
R7 = [(0, "invoke", "write", 1), (1, "invoke", "write", 2), (0, "ok", "write", 1),
      (1, "ok", "write", 2), (2, "invoke", "read", None), (2, "ok", "read", 1)]
kat("reg_R7", "cas-register", hist(*R7), True, explored=5, source=S)
kat("reg_R8", "cas-register", hist(*(R7 + [(2, "invoke", "read", None), (2, "ok", "read", 2)])),
    False, fail_idx=7, prev_ok=5, explored=5, source=S)
kat("reg_R9", "cas-register", hist((0, "invoke", "cas", [1, 2]), (0, "fail", "cas", [1, 2]),
                                   (1, "invoke", "read", None), (1, "ok", "read", None)),
    True, explored=1, source=S)

# ---- edge cases (hand-derived)
E = "edge case (hand-derived)"
kat("empty_register", "cas-register", [], True, explored=0, source=E)
kat("empty_counter", "counter", [], True, explored=0, source=E)
kat("only_invokes", "cas-register", hist((0, "invoke", "write", 1), (1, "invoke", "read", None)),
    True, explored=0, source=E)
# cas from nil with a crashed write of the expected value in flight: linearizable
kat("reg_cas_after_crashed_write", "cas-register",
    hist((0, "invoke", "write", 0), (0, "info", "write", 0), (1, "invoke", "cas", [0, 4]),
         (1, "ok", "cas", [0, 4]), (2, "invoke", "read", None), (2, "ok", "read", 4)),
    True, explored=3, source=E)
# a read observes a value whose write has not been invoked yet: invalid
kat("reg_read_from_future", "cas-register",
    hist((0, "invoke", "read", None), (0, "ok", "read", 2), (1, "invoke", "write", 2),
         (1, "ok", "write", 2)),
    False, fail_idx=1, explored=0, source=E)
kat("counter_decr", "counter",
    hist((0, "invoke", "decr", 3), (0, "ok", "decr", 3), (1, "invoke", "read", None),
         (1, "ok", "read", -3), (1, "invoke", "decr-and-get", 2), (1, "ok", "decr-and-get", [2, -5])),
    True, explored=3, source=E)
kat("counter_bad_decr_and_get", "counter",
    hist((0, "invoke", "decr", 3), (0, "ok", "decr", 3),
         (1, "invoke", "decr-and-get", 2), (1, "ok", "decr-and-get", [2, -1])),
    False, fail_idx=3, prev_ok=1, explored=1, source=E)

if __name__ == "__main__":
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
    with open(path, "w") as fh:
        json.dump(KATS, fh, indent=1)
    print(f"wrote {len(KATS)} KATs to {path}")
