"""Repro of tests/test_load_metrics.py::test_attached_roll_in_the_ingest's
first stream, batch by batch: the engine's sample against the oracle's, and
at the first difference the batch's shape and the differing entries.

usage: python scripts/repro/lm_attached.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from gen import tiny_stream  # noqa: E402
from foundationdb_amd import ConflictSet  # noqa: E402
from foundationdb_amd.conflict_set import ConflictBatch  # noqa: E402
from foundationdb_amd.load_metrics import IopsSample  # noqa: E402
from oracle.load_sample import SpecSample, roll_batch  # noqa: E402


def main():
    cs = ConflictSet(device=0)
    units = 110
    stream = list(tiny_stream(5, n_batches=14, maxlen=11))
    g, o = IopsSample(units, seed=21), SpecSample(units, seed=21)
    g.attach(cs)
    t = 0.0
    for i, (batch, now, nold) in enumerate(stream):
        packed = i % 5 == 3
        if packed:
            cs.detect_packed(batch, now, nold)
        else:
            cb = ConflictBatch(cs)
            for snap, reads, writes in batch.txns():
                cb.add_transaction(reads, writes, snap)
            cb.detect_conflicts(now, nold)
        t += 0.4
        if i % 4 == 2:
            print(f"batch {i}: T={batch.T} R={batch.R} W={batch.W} (no add)")
            continue
        off = 90 if i % 7 == 6 else 100
        before = dict(g.items())
        seq = o.seq
        ng = g.add_batch(cs, t + 1.0, offset_per_key=off)
        no = o.add_batch(batch, t + 1.0, offset_per_key=off)
        gi, oi = dict(g.items()), dict(o.items())
        print(f"batch {i}: T={batch.T} R={batch.R} W={batch.W} packed={packed} seq={seq} ng={ng} no={no} "
              f"same={gi == oi}", flush=True)
        if gi != oi:
            rolled = roll_batch(batch, 21, seq, off, units)
            print("  oracle rolled:", rolled)
            for s2 in range(max(0, seq - 3), seq + 4):
                print(f"  oracle roll at seq {s2}:", len(roll_batch(batch, 21, s2, off, units)))
            delta = {k: gi.get(k, 0) - before.get(k, 0) for k in set(gi) | set(before)}
            print("  engine added:", sorted((k, v) for k, v in delta.items() if v))
            print("  diff g-o:", sorted((k, gi.get(k, 0) - oi.get(k, 0)) for k in set(gi) | set(oi)
                                        if gi.get(k, 0) != oi.get(k, 0)))
            for k, (snap, reads, writes) in enumerate(batch.txns()):
                print("   txn", k, "writes", writes, "reads", reads)
            break
        if i % 3 == 0:
            g.poll(t)
            o.poll(t)
        if i == 8:
            g.attach(None)
            g.attach(cs)
    g.close()
    cs.close()


if __name__ == "__main__":
    main()
