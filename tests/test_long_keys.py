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
import ctypes as C
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


def tenant_stream(seed, n_batches=24, txns=4000):
    """Keys that share long prefixes per tenant (config 4's shape, smaller):
    an 8-byte tenant + a 40-byte path (two tenants share the path; one path
    differs from another only in its last byte) + 0-12 suffix bytes over a
    small alphabet, and the bare prefix, its prefix and prefix + \\x00 now
    and then -- so the directory windows and pages take prefix skips
    (common.h Dir::wsk, Pool::pskip) of 48+ bytes and the skip's 8 bytes run
    past short keys' ends.  Point writes grow the history to thousands of
    boundaries (splits, windows); wide writes erase; the window compacts."""
    rng = random.Random(seed)
    path_a = bytes(rng.choice(b"/abcdefgh") for _ in range(40))
    paths = [path_a, path_a, path_a[:-1] + b"\xff", bytes(rng.choice(b"/xyz") for _ in range(40))]
    tenants = [bytes([0, 0, 0, 0, 0, 0, 0, t]) + paths[t] for t in range(4)]

    def key(p=None):
        p = p if p is not None else rng.choice(tenants)
        u = rng.random()
        if u < 0.03:
            return p
        if u < 0.05:
            return p[:-1]
        if u < 0.07:
            return p + b"\x00"
        return p + bytes(rng.choice(b"\x00abz\xff") for _ in range(rng.randint(1, 12)))

    def rng_range(wide):
        if not wide:
            k = key()
            return (k, k + b"\x00")
        # a short range: the keys under a (a range across a tenant would erase most of the history)
        a = rng.choice(tenants) + bytes(rng.choice(b"\x00abz") for _ in range(rng.randint(2, 6)))
        return (a, a + bytes([255]) * rng.randint(1, 2))

    now, nold = 1000, 0
    for _ in range(n_batches):
        now += rng.randint(1, 5)
        if rng.random() < 0.5:
            nold = max(nold, now - rng.randint(150, 300))
        batch = []
        for _t in range(rng.randint(txns // 2, txns)):
            snap = now - rng.randint(1, 8)  # (recent snapshots: most transactions commit and write)
            reads = [rng_range(rng.random() < 0.1) for _ in range(rng.randint(0, 3))]
            writes = [rng_range(rng.random() < 0.05) for _ in range(rng.randint(0, 3))]
            batch.append((snap, reads, writes))
        yield PackedBatch.from_txns(batch), now, nold


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_prefix_skips(gpu, seed):
    """The searches' prefix skips (directory windows and pages) against the
    oracle: verdicts and the whole history after every batch, through the
    packed and per-transaction paths, a clearConflictSet and a reload of the
    history (every loaded page's skip is recomputed)."""
    cs = ConflictSet()
    c = CpuSpec()
    try:
        for i, (batch, now, nold) in enumerate(tenant_stream(seed)):
            if i == 8 and seed == 2:
                cs.clear(now - 3)
                c.clear(now - 3)
            if i == 14:  # the oracle's history into the GPU set, then on from there
                h = c.history()
                cs.load_history([k for k, _ in h], [v for _, v in h], v0=c.header_version, oldest=c.oldest_version,
                                removal_key=c.removal_key())
            vg = resolve_per_txn(cs, batch, now, nold) if i % 3 == 1 else cs.detect_packed(batch, now, nold)
            vc = c.detect_packed(batch, now, nold)
            assert np.array_equal(vg, vc), (i, np.nonzero(vg != vc)[0][:10])
            assert cs.oldest_version == c.oldest_version, i
            assert cs.removal_key() == c.removal_key(), i
            hg, hc = cs.history(), c.history()
            assert len(hg) == len(hc), (i, len(hg), len(hc))
            assert hg == hc, i
        assert len(hc) > 15000, len(hc)  # (a directory of 100+ entries: skip windows, split pages)
        out = (C.c_int64 * 3)()
        assert cs._lib.fdbcs_debug_prefix_skips(cs.handle, out, 3) == 3
        windows, pages, pending = list(out)
        assert windows > 0 and pages > 0, (windows, pages, pending)  # (the skips were in use)
    finally:
        cs.close()
        c.close()
