"""Conflict-range keys at full length (CLIENT_KNOBS->KEY_SIZE_LIMIT
10,000 + SYSTEM_KEY_SIZE_LIMIT 30,000, fdbclient/Knobs.cpp:57-58, and the
keyAfter of a 30,000-byte key: 30,001 bytes = FDBCS_MAX_KEY).

Keys share prefixes of 1,000 to 29,990 bytes and differ in a short suffix over
a tiny alphabet (so prefix relations, "", \\x00 and touching ranges all occur),
so every compare in the sort, the searches, the merge and the compaction goes
deep into the tails.  Batches alternate between the packed path and the
Resolver's per-transaction calls; one stream clears the set mid-way
(clearConflictSet, SkipList.cpp:957-959).  After every batch: verdicts, the
whole history, removalKey (a long key: the compaction's next boundary) and
oldestVersion against the oracle (oracle/cpu_spec.cpp).
"""
import random

import numpy as np
import pytest

from foundationdb_amd import ConflictBatch, ConflictSet
from foundationdb_amd import _abi
from foundationdb_amd.batch import PackedBatch
from oracle import CpuSpec

ALPHA = b"ab\x00c"


def long_stream(seed, prefix_len, n_batches=18, max_txns=30, sfx=11):
    """(PackedBatch, now, new_oldest) with keys prefix + suffix (<= FDBCS_MAX_KEY)."""
    rng = random.Random(seed)
    base = bytes(rng.choice(b"xyz/") for _ in range(prefix_len))
    alts = [base, base[:-1] + b"{", base[: prefix_len // 2]]  # a sibling prefix and a shorter one

    def key():
        p = alts[0] if rng.random() < 0.85 else rng.choice(alts)
        n = rng.randint(0, min(sfx, _abi.MAX_KEY - len(p)))
        return p + bytes(rng.choice(ALPHA) for _ in range(n))

    def rng_range():
        if rng.random() < 0.6:  # a point range on a distinct key (the history grows past the window)
            k = alts[0][: _abi.MAX_KEY - 7] + bytes(rng.choice(b"abcdefgh") for _ in range(6))
            return (k, k + b"\x00")
        while True:
            a, b = key(), key()
            if a != b:
                return (min(a, b), max(a, b))

    now, nold = 100, 0
    for _ in range(n_batches):
        now += rng.randint(1, 6)
        if rng.random() < 0.7:
            nold = max(0, now - rng.randint(10, 30))
        txns = []
        for _t in range(rng.randint(0, max_txns)):
            snap = now - rng.randint(1, 12)
            reads = [rng_range() for _ in range(rng.randint(0, 2))]
            writes = [rng_range() for _ in range(rng.randint(0, 2))]
            if rng.random() < 0.2:  # a point range [k, k\x00) of a full-length key
                k = alts[0][: _abi.MAX_KEY - 1] + b"q" * max(0, _abi.MAX_KEY - 1 - len(alts[0]))
                writes.append((k, k + b"\x00"))
            txns.append((snap, reads, writes))
        yield PackedBatch.from_txns(txns), now, nold


def resolve_per_txn(cs, batch, now, nold):
    b = ConflictBatch(cs)
    for snap, reads, writes in batch.txns():
        b.add_transaction(reads, writes, snap)
    return b.detect_conflicts(now, nold)


@pytest.mark.gpu
@pytest.mark.parametrize("prefix_len", [1000, 8000, 29990])
def test_full_length_keys(gpu, prefix_len):
    cs = ConflictSet()
    c = CpuSpec()
    longest_rk = 0
    try:
        for i, (batch, now, nold) in enumerate(long_stream(prefix_len, prefix_len)):
            if i == 9 and prefix_len == 8000:
                cs.clear(now - 4)
                c.clear(now - 4)
            vg = resolve_per_txn(cs, batch, now, nold) if i % 2 else cs.detect_packed(batch, now, nold)
            vc = c.detect_packed(batch, now, nold)
            assert np.array_equal(vg, vc), (i, np.nonzero(vg != vc)[0][:10])
            assert cs.oldest_version == c.oldest_version, i
            assert cs.removal_key() == c.removal_key(), i
            longest_rk = max(longest_rk, len(c.removal_key()))
            hg, hc = cs.history(), c.history()
            assert len(hg) == len(hc), i
            assert hg == hc, i
        assert longest_rk > 32  # a long removalKey went through the device
    finally:
        cs.close()
        c.close()
