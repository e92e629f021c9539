"""Generate the golden fixtures in tests/golden/ from the pure-Python spec.

    python tests/golden/make_golden.py

Each fixture is a JSON stream of batches: the batch's transactions (keys as
hex), (now, newOldest), and the expected verdict bytes, post-batch history
(key hex, version), removalKey and oldestVersion after every batch.

Provenance: oracle/spec.py, a restatement of SURVEY.md Appendix A.  The
reference engine cannot be executed here, so these
vectors pin regressions of the restatement and of the GPU engine against it;
they are not reference outputs ("parity unpinned").
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from gen import tiny_stream  # noqa: E402
from oracle.spec import SpecBatch, SpecConflictSet  # noqa: E402


def hx(b):
    return bytes(b).hex()


def record_stream(batches, clear_at=None):
    cs = SpecConflictSet()
    out = []
    for i, (batch, now, nold) in enumerate(batches):
        entry = {}
        if clear_at is not None and i == clear_at[0]:
            cs.clear(clear_at[1])
            entry["clear_before"] = clear_at[1]
        b = SpecBatch(cs)
        txns = batch.txns()
        for snap, reads, writes in txns:
            b.add_transaction(reads, writes, snap)
        verdict, _nc, _to = b.detect_conflicts(now, nold)
        entry.update({
            "now": now, "new_oldest": nold,
            "txns": [[snap, [[hx(x), hx(y)] for x, y in r], [[hx(x), hx(y)] for x, y in w]] for snap, r, w in txns],
            "verdict": verdict,
            "history": [[hx(k), v] for k, v in cs.history()],
            "removal_key": hx(cs.removal_key),
            "oldest": cs.oldest,
            "v0": cs.v0,
        })
        out.append(entry)
    return out


def special_cases():
    """Hand-written streams for SURVEY.md Appendix C behaviours."""
    from foundationdb_amd.batch import PackedBatch
    P = PackedBatch.from_txns
    s = []
    # C1 tooOld needs >= 1 read: blind write with an ancient snapshot commits
    # C2 tooOld compares against the previous batch's oldest
    # C3 snapshot == write version is not a conflict
    # C5 touching writes [a,k),[k,b) leave a and k at now, b at its old value
    # C6 "" as a real boundary
    s.append((P([(0, [], [(b"a", b"c")])]), 10, 0))
    s.append((P([(10, [(b"a", b"b")], [(b"", b"a")]), (9, [(b"b", b"z")], []), (0, [], [(b"x", b"y")])]), 20, 15))
    s.append((P([(5, [(b"a", b"b")], []), (0, [], [(b"a", b"k"), (b"k", b"q")]), (19, [(b"a", b"b")], [])]), 30, 16))
    s.append((P([(30, [(b"", b"\x00")], [(b"", b"\x00\x00")]), (29, [(b"j", b"l")], [])]), 40, 31))
    s.append((P([]), 50, 45))
    s.append((P([(49, [(b"a", b"b")], [(b"", b"\xff" * 20)])]), 60, 55))
    return s


def main():
    fixtures = {}
    fixtures["tiny_alphabet"] = [record_stream(list(tiny_stream(1000 + i, n_batches=12, max_txns=12)))
                                 for i in range(6)]
    fixtures["long_keys"] = [record_stream(list(tiny_stream(2000 + i, n_batches=10, max_txns=10, maxlen=40)))
                             for i in range(2)]
    fixtures["clear_mid_stream"] = [record_stream(list(tiny_stream(3000, n_batches=10, max_txns=10)),
                                                  clear_at=(5, 123))]
    fixtures["appendix_c"] = [record_stream(special_cases())]
    rng = random.Random(7)
    del rng
    for name, streams in fixtures.items():
        path = os.path.join(HERE, f"{name}.json")
        with open(path, "w") as f:
            json.dump({"source": "oracle/spec.py (SURVEY.md Appendix A restatement); parity unpinned",
                       "streams": streams}, f, separators=(",", ":"))
        print(path, sum(len(x) for x in streams), "batches")


if __name__ == "__main__":
    main()
