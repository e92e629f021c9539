"""Live ingest: from the second per-transaction batch on,
k_live_ingest encodes each batch while its transactions are still being added
(fdbcs_batch_begin launches it; TxnStage publishes progress every
FDBCS_LIVE_PUB transactions).  These tests drive the paths around it against
the CPU oracle, bit-exact on verdicts and on the full history:
  - the steady state (every batch after the first goes live),
  - a batch that outgrows the live capacities mid-batch (cancelled, ingested
    whole at detect),
  - a batch begun and abandoned (a new ConflictBatch before detect),
  - calls that need the stream while a live batch is open (history size,
    dump, a host-view detect) -- they cancel it and the batch still commits
    correctly,
  - a stream that must grow while live.
"""
import os

import numpy as np
import pytest

from foundationdb_amd import ConflictBatch, ConflictSet
from foundationdb_amd.batch import PackedBatch
from gen import mixed_stream, tiny_stream
from oracle import CpuSpec

pytestmark = pytest.mark.gpu


def same_history(g, c):
    gv, gl, go, gk = g.dump_arrays()
    cv, cl, co, ck = c.dump_arrays()
    assert len(gv) == len(cv), (len(gv), len(cv))
    if len(gv):
        assert np.array_equal(gv, cv) and np.array_equal(gl, cl)
        n = int(gl.astype(np.int64).sum())
        assert np.array_equal(gk[:n], ck[:n]), "key bytes differ"


def live_cs(pub=None, blocks=None, spec=None, timeout_us=None):
    """A conflict set whose live kernel has the given shape: FDBCS_LIVE_PUB
    (transactions per progress word), FDBCS_LIVE_BLOCKS (workgroups),
    FDBCS_LIVE_SPEC (the speculative record window), FDBCS_LIVE_TIMEOUT_US --
    read when the conflict set is made (None: the default)."""
    env = {"FDBCS_LIVE_PUB": pub, "FDBCS_LIVE_BLOCKS": blocks, "FDBCS_LIVE_SPEC": spec,
           "FDBCS_LIVE_TIMEOUT_US": timeout_us}
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is not None:
            os.environ[k] = str(v)
    try:
        return ConflictSet()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def run_batch(g, batch, now, nold):
    b = ConflictBatch(g)
    for snap, reads, writes in batch.txns():
        b.add_transaction(reads, writes, snap)
    return b.detect_conflicts(now, nold)


# (blocks, speculative window, publish cadence): the default and the shapes a
# round-4 variant build failed on (64 blocks, no speculative window: wrong
# statuses on valid input from stale host lines, fixed in f05d87a -- DESIGN §8)
LIVE_SHAPES = [(None, None, None), (64, 0, None), (64, 1, 8), (32, 1, None), (32, 0, 1000), (128, 0, 8),
               (128, 1, 1000), (2, 1, 16)]


@pytest.mark.parametrize("blocks,spec,pub", LIVE_SHAPES)
def test_live_steady_state(gpu, blocks, spec, pub):
    g = live_cs(pub, blocks, spec)
    c = CpuSpec()
    n = 0
    for batch, now, nold in mixed_stream(11, n_batches=14, max_txns=700, keyspace=4000):
        v = run_batch(g, batch, now, nold)
        assert np.array_equal(v, c.detect_packed(batch, now, nold)), n
        n += 1
    st = g.batch_stats()
    assert st["live_batches"] >= 1, st  # (mixed_stream sizes vary: some batches outgrow the caps)
    assert st["live_batches"] + st["live_cancelled"] <= n - 1
    same_history(g, c)
    g.close()


def test_live_short_keys(gpu):
    g = live_cs(8)
    c = CpuSpec()
    for batch, now, nold in tiny_stream(5, n_batches=16, max_txns=60, maxlen=11, max_reads=3, max_writes=3):
        assert np.array_equal(run_batch(g, batch, now, nold), c.detect_packed(batch, now, nold))
    assert g.batch_stats()["live_batches"] >= 1
    same_history(g, c)
    g.close()


def keyed(i, w=12):
    return b"k%0*d" % (w, i)


def txns_for(T, base, snap, width=12):
    out = []
    for t in range(T):
        k = base + 3 * t
        out.append((snap, [(keyed(k, width), keyed(k + 2, width))], [(keyed(k + 1, width), keyed(k + 1, width) + b"\x00")]))
    return out


def test_live_outgrown_cancel_and_abandon(gpu):
    g = live_cs(16)
    c = CpuSpec()
    now = 10
    # steady shape, then a batch 4x larger (cancelled mid-batch), then long keys
    # (key bytes past the caps), then back to the steady shape
    plan = [(300, 12), (300, 12), (300, 12), (1200, 12), (300, 12), (300, 200), (300, 12), (50, 12), (300, 12)]
    for i, (T, width) in enumerate(plan):
        txns = txns_for(T, 1000 * i, now - 5, width)
        pb = PackedBatch.from_txns(txns)
        b = ConflictBatch(g)
        for snap, r, w in txns:
            b.add_transaction(r, w, snap)
        v = b.detect_conflicts(now, max(0, now - 40))
        assert np.array_equal(v, c.detect_packed(pb, now, max(0, now - 40))), i
        now += 10
        if i == 4:  # a batch begun, half added, abandoned: the next batch replaces it
            ab = ConflictBatch(g)
            for snap, r, w in txns_for(100, 77_000, now - 5):
                ab.add_transaction(r, w, snap)
    st = g.batch_stats()
    assert st["live_batches"] >= 4 and st["live_cancelled"] >= 2, st
    same_history(g, c)
    g.close()


def test_live_interrupted_by_other_calls(gpu):
    """history_size / dump / a packed detect while a live batch is open: each
    cancels it (the live kernel leaves) and the open batch still detects
    correctly at the end."""
    g = live_cs(8)
    c = CpuSpec()
    now = 10
    for i in range(3):
        txns = txns_for(200, 500 * i, now - 5)
        run_pb = PackedBatch.from_txns(txns)
        b = ConflictBatch(g)
        for snap, r, w in txns:
            b.add_transaction(r, w, snap)
        assert np.array_equal(b.detect_conflicts(now, 0), c.detect_packed(run_pb, now, 0))
        now += 10
    for what in ("size", "dump", "packed"):
        txns = txns_for(200, 9000 + 700 * now, now - 5)
        b = ConflictBatch(g)
        for snap, r, w in txns[:100]:
            b.add_transaction(r, w, snap)
        if what == "size":
            assert g.history_size() == c.history_size()
        elif what == "dump":
            same_history(g, c)
        else:
            other = PackedBatch.from_txns(txns_for(30, 90_000 + now, now - 5))
            assert np.array_equal(g.detect_packed(other, now, 0), c.detect_packed(other, now, 0))
            now += 10
        for snap, r, w in txns[100:]:
            b.add_transaction(r, w, snap)
        assert np.array_equal(b.detect_conflicts(now, 0), c.detect_packed(PackedBatch.from_txns(txns), now, 0)), what
        now += 10
    same_history(g, c)
    g.close()


def test_live_stream_growth(gpu):
    """A live batch that outgrows its capacities and then its record stream
    (4 MB first allocation, ~6 MB here): cancelled at the caps, the stream
    grown after the kernel left."""
    g = live_cs(64)
    c = CpuSpec()
    now = 10
    for i, T in enumerate([2000, 2000, 5000]):
        txns = txns_for(T, 10_000 * i, now - 5, width=200)  # ~1.2 KB a transaction
        pb = PackedBatch.from_txns(txns)
        b = ConflictBatch(g)
        for snap, r, w in txns:
            b.add_transaction(r, w, snap)
        assert np.array_equal(b.detect_conflicts(now, 0), c.detect_packed(pb, now, 0)), i
        now += 10
    same_history(g, c)
    g.close()


def test_live_resolver_loop(gpu):
    """The bench's native resolver loop (fdbwl_run_resolver) goes live on
    every batch after the first and its verdicts equal the oracle's (config 2
    at 2,000 transactions)."""
    from foundationdb_amd.workload import Workload
    g = ConflictSet()
    c = CpuSpec()
    wl = Workload(2, txns=2000)
    nb = 10
    run = wl.prepare_run(0, nb)
    _, _, verdicts = run.run(g)
    for i in range(nb):
        bt, now, nold = wl.batch(i)
        assert np.array_equal(verdicts[i], c.detect_packed(bt, now, nold)), i
    st = g.batch_stats()
    assert st["live_batches"] >= nb - 2, st
    g.close()


def test_last_device_batch_after_live(gpu):
    """A live batch lays its writes out after a gap (slot 2 caps.R + 2w,
    BatchBufs::lv_wbase); fdbcs_last_device_batch hands out the view's own
    layout (writes from 2R), moving the write entries down on the call.  The
    exported view, read back from the device, holds every range of the batch
    in order: reads at 2r, 2r + 1, writes at 2R + 2w, 2R + 2w + 1."""
    import ctypes as C

    from foundationdb_amd import _abi

    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]

    def d2h(ptr, nbytes, dtype):
        out = np.empty(max(nbytes, 1), np.uint8)
        if nbytes:
            assert hip.hipMemcpy(out.ctypes.data, ptr, nbytes, 4) == 0  # (hipMemcpyDefault)
        return out[:nbytes].view(dtype)

    g = live_cs()
    lib = _abi.lib()
    checked, live_before = 0, 0
    for batch, now, nold in mixed_stream(23, n_batches=10, max_txns=400, keyspace=3000):
        run_batch(g, batch, now, nold)
        live_now = g.batch_stats()["live_batches"]
        was_live, live_before = live_now > live_before, live_now
        if not was_live:
            continue
        v = _abi.BatchView()
        _abi.check(lib.fdbcs_last_device_batch(g.handle, C.byref(v)), "fdbcs_last_device_batch")
        R, W = v.read_count, v.write_count
        slots = 2 * (R + W)
        koff = d2h(v.key_off, 8 * slots, np.uint64)
        klen = d2h(v.key_len, 4 * slots, np.uint32)
        kb = d2h(v.key_bytes, int(v.key_bytes_len), np.uint8)
        reads = [r for _, rs, _ in batch.txns() for r in rs]
        writes = [w for _, _, ws in batch.txns() for w in ws]
        assert (len(reads), len(writes)) == (R, W)

        def key(s):
            return kb[int(koff[s]):int(koff[s]) + int(klen[s])].tobytes()

        for r, (b, e) in enumerate(reads):
            assert (key(2 * r), key(2 * r + 1)) == (bytes(b), bytes(e)), ("read", r)
        for w, (b, e) in enumerate(writes):
            assert (key(2 * R + 2 * w), key(2 * R + 2 * w + 1)) == (bytes(b), bytes(e)), ("write", w)
        checked += 1
    assert checked >= 1, g.batch_stats()
    g.close()


@pytest.mark.parametrize("blocks,spec,pub", LIVE_SHAPES)
def test_live_skip_runs(gpu, blocks, spec, pub):
    """tests/test_gpu_parity.py::test_per_transaction_skip_runs on a live
    conflict set of each shape: runs of range-less transactions in one
    fdbcs_batch_skip call between the adds, verdicts and the whole history
    against the oracle after every batch."""
    import random
    g = live_cs(pub, blocks, spec)
    for seed in range(3):
        g.load_history([], [], v0=0, oldest=0, removal_key=b"")
        c = CpuSpec()
        rng = random.Random(seed)
        for batch, now, nold in mixed_stream(seed, n_batches=8, max_txns=400, keyspace=3000):
            txns = []
            for t in batch.txns():
                if rng.random() < 0.3:
                    txns += [(rng.randrange(0, now), [], [])] * rng.randint(1, 5)
                txns.append(t)
            txns += [(0, [], [])] * rng.randint(0, 3)
            vc = c.detect_packed(PackedBatch.from_txns(txns), now, nold)
            b = ConflictBatch(g)
            pending = 0
            for snap, r, w in txns:
                if not r and not w:
                    pending += 1
                    continue
                if pending:
                    b.skip(pending)
                    pending = 0
                b.add_transaction(r, w, snap)
            if pending:
                b.skip(pending)
            assert np.array_equal(b.detect_conflicts(now, nold), vc), (seed, now)
        same_history(g, c)
        c.close()
    assert g.batch_stats()["live_batches"] >= 1, g.batch_stats()
    g.close()


@pytest.mark.parametrize("pub", [8, None])
def test_live_batch_at_its_caps(gpu, pub):
    """a live batch that ends just under all four of its
    capacities (T, R, W and key bytes: the previous batch's plus a quarter,
    engine.hip live_begin) with keys longer than 17 bytes, so every key has a
    tail in the batch's tail buffer.  The buffers were sized without the
    stream's publish padding, so detectConflicts reallocated the tail buffer
    after the live kernel had written into it (keys.tail left dangling).  Now
    live_begin sizes them for the padded stream and run_batch refuses to move
    any of them."""
    g = live_cs(pub)
    c = CpuSpec()
    now = 100

    def txn(k, wlen, snap):
        key = b"key-%012d" % k + b"." * (wlen - 16)  # wlen bytes, > 17
        rk = b"key-%012d" % (k + 1) + b"r" * 8
        return (snap, [(rk, rk + b"\x00")], [(key, key + b"\x00")])

    T0 = 2000
    first = [txn(4 * t, 24, now - 5) for t in range(T0)]
    kb0 = sum(len(b) + len(e) for _, rs, ws in first for b, e in rs + ws)
    cap_t = T0 + T0 // 4 + 256  # (R = W = T here)
    cap_k = kb0 + kb0 // 4 + 65536
    T1 = cap_t - 1
    second = [txn(4 * t + 100_000, 24, now + 5) for t in range(T1)]
    kb1 = sum(len(b) + len(e) for _, rs, ws in second for b, e in rs + ws)
    extra = cap_k - 1 - kb1  # grow write keys (2 bytes of key per byte of length) up to the key cap
    i = 0
    while extra >= 2:
        snap, rs, ws = second[i]
        grow = min(extra // 2, 32 - len(ws[0][0]))  # (keys up to 32 bytes are staged whole: the most stream bytes)
        k = ws[0][0] + b"+" * grow
        second[i] = (snap, rs, [(k, k + b"\x00")])
        extra -= 2 * grow
        i += 1
    kb1 = sum(len(b) + len(e) for _, rs, ws in second for b, e in rs + ws)
    assert cap_k - 2 <= kb1 < cap_k and T1 < cap_t
    for i, txns in enumerate([first, second, first[:500]]):
        b = ConflictBatch(g)
        for snap, r, w in txns:
            b.add_transaction(r, w, snap)
        v = b.detect_conflicts(now, 0)
        assert np.array_equal(v, c.detect_packed(PackedBatch.from_txns(txns), now, 0)), i
        if i == 1:
            st = g.batch_stats()
            assert st["live_batches"] == 1 and st["live_cancelled"] == 0, st
        now += 10
    same_history(g, c)
    g.close()


def test_live_timeout_falls_back(gpu):
    """a live kernel whose adds stall past its timeout
    (here 20 ms; 8 s by default) gives up and marks the progress words; the
    batch's detectConflicts sees the mark and ingests the whole stream, so its
    verdicts and history are still exact, and the next batch goes live again."""
    import time
    g = live_cs(timeout_us=20_000)
    c = CpuSpec()
    now = 10
    for i in range(4):
        txns = txns_for(300, 1000 * i, now - 5, 20)
        b = ConflictBatch(g)
        for j, (snap, r, w) in enumerate(txns):
            if i == 2 and j == 150:
                time.sleep(0.25)  # (the kernel gives up here)
            b.add_transaction(r, w, snap)
        v = b.detect_conflicts(now, 0)
        assert np.array_equal(v, c.detect_packed(PackedBatch.from_txns(txns), now, 0)), i
        st = g.batch_stats()
        if i == 2:
            assert st["live_timeouts"] == 1 and st["live_cancelled"] >= 1, st
        now += 10
    st = g.batch_stats()
    assert st["live_timeouts"] == 1 and st["live_batches"] >= 2, st
    same_history(g, c)
    g.close()


def test_live_sort_overflow_falls_back(gpu):
    """Live batches whose keys moved away from the last batch's quantiles (a
    sort bucket overflows its staging row while the live kernel scatters):
    the overflow guard after the live kernel re-buckets them, as after the
    whole-stream ingest; verdicts and history stay exact and every batch
    after the first stays live."""
    g = live_cs(8)
    c = CpuSpec()
    now = 10
    plan = [(400, 1000), (400, 5000), (400, 9_000_000), (400, 9_001_000), (400, 20_000)]
    for i, (T, base) in enumerate(plan):
        txns = txns_for(T, base, now - 5, 14)  # (base 9 M: every key above the last batch's splitters)
        b = ConflictBatch(g)
        for snap, r, w in txns:
            b.add_transaction(r, w, snap)
        v = b.detect_conflicts(now, 0)
        assert np.array_equal(v, c.detect_packed(PackedBatch.from_txns(txns), now, 0)), i
        now += 10
    st = g.batch_stats()
    assert st["live_batches"] == len(plan) - 1 and st["sort_rebucketed"] in (0, 1), st
    same_history(g, c)
    g.close()
