"""Key-range resolvers (multi-resolver scale-out): the native proxy split vs the
oracle's restatement, the combine, and the distributed MIN all-reduce (gloo,
world_size 2) on CPU."""
import os
import random

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from foundationdb_amd.batch import PackedBatch
from foundationdb_amd.resolvers import KeyRangeResolvers, combine, uniform_bounds
from foundationdb_amd.workload import Workload
from gen import mixed_stream, tiny_stream
from oracle import CpuSpec
from oracle.spec import proxy_combine, proxy_split


def same_sub(sub, idx, ref_sub, ref_idx):
    assert list(idx) == ref_idx
    assert sub.txns() == ref_sub


@pytest.mark.parametrize("seed", range(6))
def test_split_matches_spec_tiny(seed):
    rng = random.Random(seed)
    bounds = sorted({bytes(rng.choice(b"ab\x00c") for _ in range(rng.randint(1, 2))) for _ in range(3)})
    kr = KeyRangeResolvers(bounds)
    for batch, _now, _nold in tiny_stream(seed, n_batches=10, max_txns=30):
        txns = batch.txns()
        for g in range(kr.n):
            sub, idx = kr.split(batch, g)
            same_sub(sub, idx, *proxy_split(txns, bounds, g))


def test_split_matches_spec_wide_ranges():
    bounds = [b"k000500", b"k001000", b"k001500"]
    kr = KeyRangeResolvers(bounds)
    for batch, _now, _nold in mixed_stream(3, n_batches=4, max_txns=200, wide=0.3):
        txns = batch.txns()
        for g in range(kr.n):
            sub, idx = kr.split(batch, g)
            same_sub(sub, idx, *proxy_split(txns, bounds, g))


def test_owner_and_bounds():
    kr = KeyRangeResolvers([b"b", b"d"])
    assert [kr.owner(k) for k in [b"", b"a", b"b", b"c", b"d", b"zz"]] == [0, 0, 1, 1, 2, 2]
    with pytest.raises(ValueError):
        KeyRangeResolvers([b"d", b"b"])
    assert uniform_bounds(4) == [bytes([64, 0, 0, 0, 0, 0, 0, 0]), bytes([128] + [0] * 7), bytes([192] + [0] * 7)]


def test_combine_matches_spec():
    rng = random.Random(1)
    T = 50
    parts = []
    for _ in range(3):
        idx = sorted(rng.sample(range(T), 20))
        parts.append(([rng.choice([0, 1, 2]) for _ in idx], idx))
    assert list(combine(T, [(np.array(v), np.array(i)) for v, i in parts])) == proxy_combine(T, parts)


def run_resolvers_cpu(batches, bounds):
    """N oracle resolvers fed by the native split; returns combined verdicts per batch."""
    kr = KeyRangeResolvers(bounds)
    res = [CpuSpec() for _ in range(kr.n)]
    out = []
    for batch, now, nold in batches:
        parts = []
        for g in range(kr.n):
            sub, idx = kr.split(batch, g)
            parts.append((res[g].detect_packed(sub, now, nold), idx))
        out.append(combine(batch.T, parts))
    return out


def test_single_resolver_is_the_conflict_set():
    batches = list(mixed_stream(7, n_batches=6, max_txns=150))
    one = run_resolvers_cpu(batches, [])
    c = CpuSpec()
    for (batch, now, nold), v in zip(batches, one):
        assert np.array_equal(v, c.detect_packed(batch, now, nold))


def _rank_main(rank, world, port, bounds, ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kr = KeyRangeResolvers(bounds)
    res = CpuSpec()
    wl = Workload(2, txns=400)
    got = []
    for i in range(5):
        batch, now, nold = wl.batch(i)
        sub, idx = kr.split(batch, rank)
        v = res.detect_packed(sub, now, nold)
        full = torch.full((batch.T,), 2, dtype=torch.uint8)
        full[torch.from_numpy(idx.astype(np.int64))] = torch.from_numpy(v)
        dist.all_reduce(full, op=dist.ReduceOp.MIN)
        got.append(full.numpy().copy())
    if rank == 0:
        ret.put([g.tolist() for g in got])
    dist.destroy_process_group()


def test_distributed_min_combine_gloo():
    """world_size 2 over gloo: each rank is one key-range resolver; the MIN
    all-reduce of scattered verdicts equals the single-process proxy combine."""
    bounds = uniform_bounds(2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.Random(os.getpid()).randint(0, 2000)
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, bounds, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    wl = Workload(2, txns=400)
    want = run_resolvers_cpu([wl.batch(i) for i in range(5)], bounds)
    for g, w in zip(got, want):
        assert g == w.tolist()
