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


def live_cs(pub=None):
    old = os.environ.get("FDBCS_LIVE_PUB")
    if pub is not None:
        os.environ["FDBCS_LIVE_PUB"] = str(pub)
    try:
        return ConflictSet()
    finally:
        if pub is not None:
            if old is None:
                del os.environ["FDBCS_LIVE_PUB"]
            else:
                os.environ["FDBCS_LIVE_PUB"] = old


def run_batch(g, batch, now, nold):
    b = ConflictBatch(g)
    for snap, reads, writes in batch.txns():
        b.add_transaction(reads, writes, snap)
    return b.detect_conflicts(now, nold)


@pytest.mark.parametrize("pub", [None, 8, 1000])
def test_live_steady_state(gpu, pub):
    g = live_cs(pub)
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
