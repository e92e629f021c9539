"""fdbcs_sharded (include/fdbcs.h): one exact Resolver over G GPUs behind the
C ABI -- the HIP engine, the protocol's exchanges and device-side carry-ins /
compaction plan inside libfdbcs (SURVEY.md §8e protocols A and B).  Under B
each rank's per-transaction adds drop the ranges outside its keys inside
libfdbcs, its packed batches are the keep-all split, and the overlap edges
travel in exchange 1's counts + one all-gather.

On the one-GPU test box the ranks share GPU 0 and exchange through host
collectives over torch.distributed gloo (fdbcs_comm_ops); the RCCL path is
the same code with the exchanges on the stream (bench.py --gpus N).  After
every batch, every rank's verdicts, the concatenation of the ranks'
histories, removalKey (read from the rank that owns it) and oldestVersion
must equal one conflict set's (oracle/cpu_spec.cpp).
"""
import os
import random

import numpy as np
import pytest
import torch.multiprocessing as mp

from gen import mixed_stream, rand_key, tiny_stream
from oracle import CpuSpec


def _streams(kind, seed):
    if kind == "tailgc":  # long keys, many times the tail arena over the stream (tests/test_tail_gc.py)
        from test_tail_gc import long_key_stream
        return list(long_key_stream(seed, 240))
    if kind == "tiny":
        return list(tiny_stream(seed, n_batches=25, maxlen=3))
    if kind == "long":
        return list(tiny_stream(seed, n_batches=20, maxlen=40))
    return list(mixed_stream(seed, n_batches=8, max_txns=400, keyspace=3000))


def _rank(rank, world, port, bounds, kind, seed, q, protocol="a", edge_cap=None, sh_ecap=None):
    if edge_cap:  # (a tiny first edge list: every shard searches again into a larger one)
        os.environ["FDBCS_TEST_EDGE_CAP"] = str(edge_cap)
    if sh_ecap:  # (a tiny edge exchange: the batch runs from exchange 1 again with a larger one)
        os.environ["FDBCS_TEST_SH_ECAP"] = str(sh_ecap)
    import torch
    import torch.distributed as dist

    from foundationdb_amd.sharded import ShardedResolver

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        arena = (4 << 20) if kind == "tailgc" else 0
        sh = ShardedResolver(bounds, rank, world, device=0, protocol=protocol, tail_arena_bytes=arena)
        out = []
        halves = set()
        for i, (batch, now, nold) in enumerate(_streams(kind, seed)):
            if kind == "tiny" and i == 12:
                sh.clear(now - 5)  # clearConflictSet mid-stream (SkipList.cpp:957-959)
            if i % 3 == 1:  # the Resolver's per-transaction calls
                v = sh.detect_txns(batch.txns(), now, nold)
            else:
                v = sh.detect_packed(batch, now, nold)
            owner = sh.removal_key_owner()
            rk = sh.local.removal_key() if owner == rank else None
            if kind == "tailgc":  # the arena stays at its initial size; both halves get used
                st = sh.local.batch_stats()
                assert st["tail_arena_bytes"] == arena, (i, st)
                halves.add(st["tail_half"])
                if i % 40 != 39:  # (histories compared every 40th batch)
                    out.append((v.tolist(), None, owner, rk, sh.local.oldest_version))
                    continue
            out.append((v.tolist(), sh.history(), owner, rk, sh.local.oldest_version))
        if kind == "tailgc":
            assert halves == {0, 1}, f"rank {rank} never freed a half"
        sh.close()
        q.put((rank, out))
    except Exception as e:  # (report, so the parent does not wait for the timeout)
        q.put((rank, repr(e)))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", ["a", "b"])
@pytest.mark.parametrize("world,kind", [(2, "tiny"), (3, "tiny"), (2, "long"), (2, "mixed"), (3, "mixed")])
def test_sharded_abi_equals_one_conflict_set(gpu, world, kind, protocol, edge_cap=None, sh_ecap=None):
    rng = random.Random(world * 31 + len(kind))
    if kind == "mixed":
        bounds = sorted({b"k%06d" % rng.randrange(1, 3000) for _ in range(world - 1)})
    else:
        alpha = b"ab\x00c"
        ks = set()
        while len(ks) < world - 1:
            ks.add(rand_key(rng, 3, alpha))
        bounds = sorted(ks)
    assert len(bounds) == world - 1
    seed = 4321 + world + len(kind)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.Random(os.getpid() * 13 + world + len(kind) + 7 * ord(protocol[0])).randint(0, 3000)
    procs = [ctx.Process(target=_rank, args=(r, world, port, bounds, kind, seed, q, protocol, edge_cap, sh_ecap))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(got[r], str), f"rank {r}: {got[r]}"
    c = CpuSpec()
    for i, (batch, now, nold) in enumerate(_streams(kind, seed)):
        if kind == "tiny" and i == 12:
            c.clear(now - 5)
        vc = c.detect_packed(batch, now, nold).tolist()
        hist = []
        owners = set()
        for r in range(world):
            v, h, owner, rk, old = got[r][i]
            assert v == vc, (i, r, np.nonzero(np.array(v) != np.array(vc))[0][:10])
            assert old == c.oldest_version, (i, r)
            owners.add(owner)
            if rk is not None:
                assert rk == c.removal_key(), (i, r)
            hist = None if h is None or hist is None else hist + h
        assert len(owners) == 1, (i, owners)  # every rank agrees on removalKey's owner
        if owners == {-1}:
            assert c.removal_key() == b"", i
        if hist is not None:
            assert hist == c.history(), i
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", ["a", "b"])
def test_sharded_abi_tail_arena_gc(gpu, protocol):
    """Long keys (43-100 B) many times the 4 MB tail arena over the stream,
    split across two ranks in the middle of their random suffixes: every
    rank's arena stays at its initial size and both halves get used."""
    import test_tail_gc
    bounds = [test_tail_gc.PREFIX + b"\x80"]
    seed = 77
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.Random(os.getpid() * 17 + ord(protocol)).randint(0, 3000)
    procs = [ctx.Process(target=_rank, args=(r, 2, port, bounds, "tailgc", seed, q, protocol)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(got[r], str), f"rank {r}: {got[r]}"
    c = CpuSpec()
    for i, (batch, now, nold) in enumerate(_streams("tailgc", seed)):
        vc = c.detect_packed(batch, now, nold).tolist()
        hist = []
        for r in range(2):
            v, h, _owner, _rk, _old = got[r][i]
            assert v == vc, (i, r)
            hist = None if h is None or hist is None else hist + h
        if hist is not None:
            assert hist == c.history(), i
    c.close()


@pytest.mark.gpu
def test_sharded_abi_protocol_b_edge_overflow(gpu):
    """Protocol B with a 3-pair first edge list: the overlapping mixed stream
    overflows it on some rank, every rank searches again (exchange 1
    repeats) and the edges travel in the all-gather."""
    test_sharded_abi_equals_one_conflict_set(gpu, 3, "mixed", "b", edge_cap=3)


@pytest.mark.gpu
@pytest.mark.parametrize("world,kind", [(3, "mixed"), (2, "tiny")])
def test_sharded_abi_protocol_b_short_exchange(gpu, world, kind):
    """Protocol B enqueues a whole batch without a host read: the edge
    all-gather has a fixed capacity per shard (here 2 pairs).  A batch whose
    lists do not fit is marked on every rank; its merge, plan and compaction
    leave the history as it was, and the batch runs from exchange 1 again with
    a larger capacity.  Verdicts, histories, removalKey
    and oldestVersion as one conflict set's after every batch."""
    test_sharded_abi_equals_one_conflict_set(gpu, world, kind, "b", sh_ecap=2)


def _burst_stream(seed):
    """One batch dense with overlapping ranges (hundreds of overlap edges per
    shard), then sparse point batches over a wide key space (almost none)."""
    from gen import PackedBatch
    rng = random.Random(seed)
    now = 1000
    for i in range(24):
        now += 100
        txns = []
        n, space, wide = (600, 400, 0.5) if i == 1 else (60, 200000, 0.0)
        for _t in range(n):
            def rr():
                a = rng.randrange(space)
                b = min(space, a + rng.randint(1, space // 4)) if rng.random() < wide else a + 1
                return (b"k%07d" % a, b"k%07d" % b)
            txns.append((now - rng.randint(1, 90), [rr() for _ in range(3)], [rr() for _ in range(2)]))
        yield PackedBatch.from_txns(txns), now, now - 500


def _burst_rank(rank, world, port, bounds, q):
    os.environ["FDBCS_TEST_SH_ECAP"] = "64"
    os.environ["FDBCS_SH_ECAP_WINDOW"] = "4"
    import torch
    import torch.distributed as dist

    from foundationdb_amd.sharded import ShardedResolver

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        sh = ShardedResolver(bounds, rank, world, device=0, protocol="b")
        out = []
        for i, (batch, now, nold) in enumerate(_burst_stream(5)):
            v = sh.detect_txns(batch.txns(), now, nold) if i % 2 else sh.detect_packed(batch, now, nold)
            out.append((v.tolist(), sh.history(), sh.exchange_stats()))
        sh.close()
        q.put((rank, out))
    except Exception as e:
        q.put((rank, repr(e)))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_abi_protocol_b_exchange_decays_after_burst(gpu):
    """protocol B's edge exchange capacity grows on a
    burst batch and returns to its floor once a window of batches (4 here)
    needed at most half of it, on every rank at the same batch -- so one
    burst no longer raises every later batch's all-gather.  Verdicts and
    histories as one conflict set's after every batch."""
    world = 2
    bounds = [b"k0000200"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.Random(os.getpid() * 19 + 3).randint(0, 3000)
    procs = [ctx.Process(target=_burst_rank, args=(r, world, port, bounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(got[r], str), f"rank {r}: {got[r]}"
    c = CpuSpec()
    for i, (batch, now, nold) in enumerate(_burst_stream(5)):
        vc = c.detect_packed(batch, now, nold).tolist()
        hist = []
        for r in range(world):
            v, h, _st = got[r][i]
            assert v == vc, (i, r)
            hist += h
        assert hist == c.history(), i
        assert got[0][i][2]["ecap"] == got[1][i][2]["ecap"], (i, got[0][i][2], got[1][i][2])
    c.close()
    st = [got[0][i][2] for i in range(len(got[0]))]
    caps = [x["ecap"] for x in st]
    assert st[1]["retries"] >= 1 and max(caps) > 64, st[:3]  # the burst ran short and grew the exchange
    assert caps[-1] <= 128 and st[-1]["shrinks"] >= 1, caps  # and it came back down
    assert max(x["last_max"] for x in st[8:]) < 64, st[8:]


@pytest.mark.gpu
def test_sharded_abi_rccl_one_rank(gpu):
    """The RCCL path (exchanges on the engine's stream) with one rank: the same
    stream as one conflict set, through both the packed and per-txn calls."""
    from foundationdb_amd.sharded import ShardedResolver
    sh = ShardedResolver([], 0, 1, device=0, comm_id=ShardedResolver.unique_id())
    c = CpuSpec()
    for i, (batch, now, nold) in enumerate(_streams("mixed", 99)):
        v = sh.detect_txns(batch.txns(), now, nold) if i % 2 else sh.detect_packed(batch, now, nold)
        assert np.array_equal(v, c.detect_packed(batch, now, nold)), i
        assert sh.history() == c.history(), i
        assert sh.local.removal_key() == c.removal_key(), i
    sh.close()
    c.close()


def _abort_init_child():
    """Rank 0 of a 2-rank RCCL communicator whose rank 1 never joins: its
    fdbcs_sharded_comm_init waits (non-blocking init, polled) until another
    thread calls fdbcs_sharded_abort; then it fails, the handle is destroyed
    cleanly, and a later call on it is refused."""
    import ctypes as C
    import threading
    import time

    import torch

    from foundationdb_amd import _abi
    from foundationdb_amd.sharded import ShardedResolver

    torch.cuda.set_device(0)
    lib = _abi.lib()
    kb = np.frombuffer(b"m\0", np.uint8).copy()
    offs = np.zeros(1, np.uint64)
    lens = np.ones(1, np.uint32)
    cfg = _abi.Config(device=0, max_history=1 << 12, tail_arena_bytes=0)
    h = C.c_void_p()
    assert lib.fdbcs_sharded_create(C.byref(h), 0, 2, kb.ctypes.data, offs.ctypes.data, lens.ctypes.data, 0,
                                    C.byref(cfg), None, None) == 0
    cid = (C.c_uint8 * _abi.COMM_ID_BYTES).from_buffer_copy(ShardedResolver.unique_id())
    res = {}

    def init():
        res["rc"] = lib.fdbcs_sharded_comm_init(h, cid)

    t = threading.Thread(target=init)
    t.start()
    time.sleep(1.0)
    assert t.is_alive(), f"init returned without its peer: {res}"
    assert lib.fdbcs_sharded_abort(h) == 0
    t.join(timeout=30)
    assert not t.is_alive(), "fdbcs_sharded_abort did not end the pending initialisation"
    assert res["rc"] != 0
    assert lib.fdbcs_sharded_batch_begin(h) == 0  # (local state only)
    out = np.zeros(1, np.uint8)
    assert lib.fdbcs_sharded_batch_detect(h, 10, 0, out.ctypes.data) != 0  # exchanges refused after the abort
    lib.fdbcs_sharded_destroy(h)
    print("ABORT_OK", flush=True)


@pytest.mark.gpu
def test_sharded_abi_rccl_abort_during_init(gpu):
    """fdbcs_sharded_abort from another thread while the rank waits
    in RCCL for a peer that never joins (a rank whose own init failed)."""
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = [%r, %r]; import test_sharded_abi as t; t._abort_init_child()"
            % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ABORT_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
