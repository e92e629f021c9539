"""Exact sharded mode (SURVEY.md §8e protocols A and B): one Resolver over G shards.

Protocol A: every shard receives the whole batch.  Protocol B (sparse=True):
each shard receives only the ranges intersecting its keys, finds the overlap
edges among them, and the edge lists are all-gathered before the decision.

The concatenated shard histories, the verdicts, removalKey and oldestVersion
must equal ONE conflict set's (the oracle) after every batch -- the north
star's "result matches a single-resolver reference exactly".

CPU tests drive the host protocol (plan_compaction, carry-ins, removalKey
broadcast; in-process and over gloo with world_size 2 and 3) with the CPU
shard model (tests/shard_model.py).  GPU tests drive the HIP engines through
the C ABI (fdbcs_shard_*), G shards on one device.
"""
import os
import random

import numpy as np
import pytest
import torch.multiprocessing as mp

from foundationdb_amd.resolvers import uniform_bounds
from foundationdb_amd.sharded import ShardedConflictSet, carry_ins, plan_compaction
from gen import ALPHA, mixed_stream, rand_key, tiny_stream
from oracle import CpuSpec
from shard_model import ModelShard


def random_bounds(rng, G, maxlen, alpha=ALPHA):
    ks = set()
    while len(ks) < G - 1:
        ks.add(rand_key(rng, maxlen, alpha))
    return sorted(ks)


def check_step(sh, c, batch, now, nold, history=True):
    vs = sh.detect_packed(batch, now, nold)
    vc = c.detect_packed(batch, now, nold)
    assert np.array_equal(vs, vc), (np.nonzero(vs != vc)[0][:10], vs[:20], vc[:20])
    assert sh.oldest_version == c.oldest_version
    if history:
        assert sh.history() == c.history()
        assert sh.removal_key() == c.removal_key()


# ------------------------------------------------------------------ CPU ----

def test_plan_compaction_cuts_the_global_window():
    # shards of 3, 0, 4 boundaries; removalKey's first hit in shard 0 at index 2
    infos = [(3, 2, 50), (0, 0, -(1 << 63)), (4, 0, 70)]
    parts, owner = plan_compaction(infos, 0)  # window = 10 boundaries: all 5 from global 2
    assert parts == [(2, 3, 1, 0), (0, 0, 0, 0), (0, 4, 0, 50)]
    assert owner is None  # the scan reached the end: removalKey wraps to ""
    parts, owner = plan_compaction([(30, 25, 9), (20, 0, 8)], 0)
    assert parts == [(25, 30, 1, 0), (0, 5, 0, 9)]
    assert owner == (1, 5)
    parts, owner = plan_compaction([(3, 3, 1), (2, 2, 2)], 4)  # nothing >= removalKey anywhere
    assert owner is None and all(p[0] == p[1] for p in parts)


def test_carry_ins_skip_empty_shards():
    assert carry_ins(7, [(2, 11), (0, 0), (1, 13), (0, 0)]) == [7, 11, 11, 13]


@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("G", [1, 2, 3, 5])
def test_model_shards_equal_one_conflict_set(G, sparse):
    for seed in range(12):
        rng = random.Random(seed * 7 + G)
        maxlen = rng.choice([2, 3, 6])
        sh = ShardedConflictSet(random_bounds(rng, G, maxlen), devices=[-1] * G, shard_factory=ModelShard,
                                sparse=sparse)
        c = CpuSpec()
        for batch, now, nold in tiny_stream(seed * 31 + G, n_batches=25, maxlen=maxlen):
            check_step(sh, c, batch, now, nold)


@pytest.mark.parametrize("sparse", [False, True])
def test_model_shards_bounds_at_written_keys_and_clear(sparse):
    """Splitters that are themselves written/read keys (e = s_g ends), clearConflictSet mid-stream."""
    sh = ShardedConflictSet([b"a", b"b", b"b\x00"], devices=[-1] * 4, shard_factory=ModelShard, sparse=sparse)
    c = CpuSpec()
    for i, (batch, now, nold) in enumerate(tiny_stream(99, n_batches=40, maxlen=3)):
        if i == 20:
            sh.clear(now - 3)
            c.clear(now - 3)
        check_step(sh, c, batch, now, nold)


@pytest.mark.parametrize("sparse", [False, True])
def test_model_shards_mixed_streams(sparse):
    for seed in range(2):
        sh = ShardedConflictSet([b"k001000", b"k002500", b"k002500\x00"], devices=[-1] * 4,
                                shard_factory=ModelShard, sparse=sparse)
        c = CpuSpec()
        for batch, now, nold in mixed_stream(seed, n_batches=8, max_txns=120, keyspace=4000):
            check_step(sh, c, batch, now, nold)


def _dist_rank(rank, world, port, bounds, seed, maxlen, sparse, q, edge_inline=1024):
    import torch.distributed as dist

    from foundationdb_amd.sharded import DistShardedConflictSet

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = DistShardedConflictSet(bounds, rank, world, device=-1, shard_factory=ModelShard, sparse=sparse,
                                edge_inline=edge_inline)
    out = []
    for batch, now, nold in tiny_stream(seed, n_batches=25, maxlen=maxlen):
        v = sh.detect_packed(batch, now, nold)
        out.append((v.tolist(), sh.history(), sh.removal_key(), sh.oldest_version))
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,maxlen,sparse,ei", [(2, 3, False, 1024), (3, 3, False, 1024), (2, 40, False, 1024),
                                                    (2, 3, True, 1024), (3, 3, True, 1024), (2, 40, True, 1024),
                                                    (3, 3, True, 1)])
def test_dist_sharded_gloo(world, maxlen, sparse, ei):
    """world_size 2/3 over gloo: one shard per rank; every rank's verdicts, the
    concatenation of the ranks' histories and removalKey equal one conflict set's
    (maxlen 40: removalKeys longer than the all-gather's inline 32 bytes;
    ei 1: protocol B edge lists too long to ride in exchange 1)."""
    rng = random.Random(world)
    bounds = random_bounds(rng, world, 3)
    seed = 1234 + world + maxlen
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.Random(os.getpid() * 7 + world).randint(0, 3000)
    procs = [ctx.Process(target=_dist_rank, args=(r, world, port, bounds, seed, maxlen, sparse, q, ei)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = CpuSpec()
    for i, (batch, now, nold) in enumerate(tiny_stream(seed, n_batches=25, maxlen=maxlen)):
        vc = c.detect_packed(batch, now, nold).tolist()
        hist = []
        for r in range(world):
            v, h, rk, old = got[r][i]
            assert v == vc, (i, r)
            assert rk == c.removal_key() and old == c.oldest_version
            hist += h
        assert hist == c.history(), i


# ------------------------------------------------------------------ GPU ----

@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("maxlen", [3, 11, 40])
def test_gpu_shards_tiny_streams(gpu, maxlen, sparse):
    for seed in range(8):
        rng = random.Random(seed * 5 + maxlen)
        G = rng.choice([2, 3, 4])
        sh = ShardedConflictSet(random_bounds(rng, G, min(maxlen, 4)), max_history=1 << 14, sparse=sparse)
        c = CpuSpec()
        try:
            for batch, now, nold in tiny_stream(seed * 13 + maxlen, n_batches=25, maxlen=maxlen):
                check_step(sh, c, batch, now, nold)
        finally:
            sh.close()


def first_batch_cases():
    """Shard 0 empty, and a committed write beginning at "" in its first batch
    (SkipList.cpp:511-522): the state of round
    3's one-off failure of test_gpu_shards_tiny_streams[11-False] (seed 0:
    bounds [cbac, ccbb], batch 0 at now=14 -- the oracle's history
    [("", 14), ("ccab\\0\\0", 0)], the GPU's without the begin at "").  Its
    batch, plus hand-built writes from "" ending inside shard 0, exactly at the
    split key and beyond it."""
    batch, now, nold = next(tiny_stream(11, n_batches=1, maxlen=11))
    yield [b"cbac", b"ccbb"], batch, now, nold
    from foundationdb_amd.batch import PackedBatch
    for end in (b"a", b"m", b"m\x00", b"zz"):
        txns = [(5, [], [(b"", end)]), (5, [(b"", b"\x00")], [(b"\x00", b"b")])]
        yield [b"m"], PackedBatch.from_txns(txns), 14, 0


@pytest.mark.parametrize("sparse", [False, True])
def test_model_shards_first_batch_from_empty_key(sparse):
    for bounds, batch, now, nold in first_batch_cases():
        sh = ShardedConflictSet(bounds, devices=[-1] * (len(bounds) + 1), shard_factory=ModelShard, sparse=sparse)
        check_step(sh, CpuSpec(), batch, now, nold)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_gpu_shards_first_batch_from_empty_key(gpu, sparse):
    """Regression: fresh shard engines -- one set per round,
    so every round starts from freshly allocated device memory -- take a
    first batch whose committed write begins at "" while shard 0 is empty."""
    for rnd in range(12):
        for bounds, batch, now, nold in first_batch_cases():
            sh = ShardedConflictSet(bounds, max_history=1 << 14, sparse=sparse)
            try:
                check_step(sh, CpuSpec(), batch, now, nold)
            finally:
                sh.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_gpu_shards_bounds_at_keys_and_clear(gpu, sparse):
    sh = ShardedConflictSet([b"a", b"b", b"b\x00"], max_history=1 << 14, sparse=sparse)
    c = CpuSpec()
    try:
        for i, (batch, now, nold) in enumerate(tiny_stream(99, n_batches=40, maxlen=3)):
            if i == 20:
                sh.clear(now - 3)
                c.clear(now - 3)
            check_step(sh, c, batch, now, nold)
    finally:
        sh.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_gpu_shards_mixed_streams(gpu, sparse):
    sh = ShardedConflictSet([b"k001000", b"k002500", b"k002500\x00"], max_history=1 << 16, sparse=sparse)
    c = CpuSpec()
    try:
        for batch, now, nold in mixed_stream(3, n_batches=12, max_txns=600, keyspace=5000):
            check_step(sh, c, batch, now, nold)
    finally:
        sh.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("G", [2, 4])
def test_gpu_shards_config2(gpu, G, sparse):
    """Config 2's shape (5R+2W, uniform 16-byte keys) split over G uniform key slices."""
    from foundationdb_amd.workload import Workload

    sh = ShardedConflictSet(uniform_bounds(G), sparse=sparse)
    c = CpuSpec()
    wl = Workload(2, txns=1500)
    try:
        for i in range(12):
            batch, now, nold = wl.batch(i)
            check_step(sh, c, batch, now, nold, history=(i % 4 == 3))
    finally:
        sh.close()


@pytest.mark.gpu
def test_gpu_shards_protocol_b_zipf_and_large(gpu):
    """Protocol B with Zipf hot keys (many overlap edges, duplicated across
    shards) and a batch past LARGE_T (merge sort in every shard)."""
    from foundationdb_amd.workload import Workload

    sh = ShardedConflictSet(uniform_bounds(3), sparse=True)
    c = CpuSpec()
    try:
        wl = Workload(3, txns=3000)
        for i in range(6):
            batch, now, nold = wl.batch(i)
            check_step(sh, c, batch, now, nold, history=(i % 3 == 2))
        wl = Workload(2, txns=80_000)
        for i in range(6, 8):
            batch, now, nold = wl.batch(i)
            check_step(sh, c, batch, now, nold, history=(i == 7))
    finally:
        sh.close()


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [True, False])
def test_dist_sharded_hip_engines(gpu, sparse):
    """The bench's N > 1 path -- DistShardedConflictSet, one HIP engine per
    process, exchanges over torch.distributed (gloo; both ranks on this GPU)
    -- at the bench's batch size past the point where a 2-process rehearsal
    once faulted (~50 batches), against one oracle conflict set: verdicts every
    batch, history sizes at the end."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "dist_hip_verify.py"), "2", "80", "10000",
                        "1" if sparse else "0"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
