"""Tail-arena GC (kernels_hist.hip move_tail / k_win_dir): keys longer than 17
bytes keep their bytes 17.. in an arena of two halves; the compaction window
moves the survivors' tails out of the old half, and a sweep that covered the
whole history frees it -- in the exact sharded modes too, where a shard frees
its old half once the global sweep has passed over all of its keys.  A long-key stream whose total tail bytes are many
times the arena must then run in the initial arena, bit-exact against the
oracle."""
import random

import numpy as np
import pytest

from foundationdb_amd.batch import PackedBatch
from oracle import CpuSpec

PREFIX = b"/tenant/0007/app/orders/by-customer/"  # 36 shared bytes: tails differ only past them


def long_key_stream(seed, n_batches, txns=200):
    rng = random.Random(seed)
    now = 10_000

    def key():
        return PREFIX + bytes(rng.randrange(256) for _ in range(rng.randint(24, 64)))

    for _ in range(n_batches):
        now += 100
        out = []
        for _t in range(txns):
            reads, writes = [], []
            for _ in range(2):
                k = key()
                reads.append((k, k + b"\x00") if rng.random() < 0.7 else (k, k + b"\xff"))
            for _ in range(2):
                k = key()
                writes.append((k, k + b"\x00"))
            out.append((now - rng.randint(1, 250), reads, writes))
        yield PackedBatch.from_txns(out), now, now - 300  # a short window: boundaries die within 3 batches


@pytest.mark.gpu
def test_long_key_stream_stays_in_the_initial_arena(gpu):
    from foundationdb_amd import ConflictSet
    arena = 4 << 20
    g = ConflictSet(device=0, tail_arena_bytes=arena)
    c = CpuSpec()
    halves = set()
    for i, (b, now, nold) in enumerate(long_key_stream(5, 400)):
        v = g.detect_packed(b, now, nold)
        assert np.array_equal(v, c.detect_packed(b, now, nold)), i
        st = g.batch_stats()
        halves.add(st["tail_half"])
        assert st["tail_arena_bytes"] == arena, f"batch {i}: the tail arena grew: {st} halves seen {halves}"
        if i % 25 == 24:
            assert g.history() == c.history(), i
            assert g.removal_key() == c.removal_key(), i
    # every write adds two boundaries with tails of 43..83 bytes: ~20 MB over the stream, 5x the arena
    new_tail_bytes = 400 * 200 * 2 * 2 * 43
    assert new_tail_bytes > 3 * arena
    assert halves == {0, 1}, "no sweep freed a half"
    assert g.history() == c.history()
    g.close()
    c.close()


def check_shards_in_arena(stats_per_shard, arena, halves, i):
    for g, st in enumerate(stats_per_shard):
        halves[g].add(st["tail_half"])
        assert st["tail_arena_bytes"] == arena, f"batch {i} shard {g}: the tail arena grew: {st}"


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_sharded_long_key_stream_stays_in_the_initial_arena(gpu, sparse):
    """Two shards split in the middle of the random suffixes (the Python
    protocol, fdbcs_shard_compact's explicit windows; protocol A and B)."""
    from foundationdb_amd.sharded import ShardedConflictSet
    arena = 4 << 20
    sh = ShardedConflictSet([PREFIX + b"\x80"], max_history=1 << 20, sparse=sparse, tail_arena_bytes=arena)
    c = CpuSpec()
    halves = [set(), set()]
    for i, (b, now, nold) in enumerate(long_key_stream(6, 300)):
        v = sh.detect_packed(b, now, nold)
        assert np.array_equal(v, c.detect_packed(b, now, nold)), i
        check_shards_in_arena([x.cs.batch_stats() for x in sh.shards], arena, halves, i)
        if i % 25 == 24:
            assert sh.history() == c.history(), i
            assert sh.removal_key() == c.removal_key(), i
    assert all(h == {0, 1} for h in halves), f"a shard never freed a half: {halves}"
    assert sh.history() == c.history()
    c.close()
