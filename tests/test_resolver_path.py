"""GPU parity of the Resolver's own path: ConflictBatch + T x addTransaction +
detectConflicts (Resolver.actor.cpp:140-153) through fdbcs_batch_begin /
fdbcs_batch_add / fdbcs_batch_detect -- the per-transaction staging stream,
its chunked H2D copies and the device unpack (engine.hip, k_unpack) -- against
the CPU oracle, bit-exact on verdicts and on the full history.
"""
import os

import numpy as np
import pytest

from foundationdb_amd import ConflictBatch, ConflictSet, FdbcsError
from foundationdb_amd import _abi
from foundationdb_amd.workload import Workload
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
    assert g.removal_key() == c.removal_key()
    assert g.oldest_version == c.oldest_version


def make_cs(chunk):
    """A conflict set whose staging stream flushes every `chunk` bytes (None: default)."""
    old = os.environ.get("FDBCS_STAGE_CHUNK")
    if chunk is not None:
        os.environ["FDBCS_STAGE_CHUNK"] = str(chunk)
    try:
        return ConflictSet()
    finally:
        if chunk is not None:
            if old is None:
                del os.environ["FDBCS_STAGE_CHUNK"]
            else:
                os.environ["FDBCS_STAGE_CHUNK"] = old


@pytest.mark.parametrize("cfg,T,nb,chunk", [(2, 2000, 12, None), (2, 2000, 6, 4096), (1, 2500, 10, None),
                                            (3, 1500, 10, 65536), (4, 400, 8, 8192), (5, 1_000_000, 2, None)])
def test_resolver_loop_matches_oracle(gpu, cfg, T, nb, chunk):
    """The bench's timed loop (native: fdbwl_run_resolver) against cpu_spec.
    (Config 5: 10^6 addTransaction calls per batch -- the staging stream grows
    to ~300 MB mid-batch and the large-batch pipeline runs on the staged
    ingest.)"""
    g = make_cs(chunk)
    c = CpuSpec()
    wl = Workload(cfg, txns=T)
    run = wl.prepare_run(0, nb)
    us, add_us, verdicts = run.run(g)
    assert us.shape == (nb,) and np.all(us > 0) and np.all(add_us <= us)
    for i in range(nb):
        b, now, nold = wl.batch(i)
        vc = c.detect_packed(b, now, nold)
        assert np.array_equal(verdicts[i], vc), (i, np.nonzero(verdicts[i] != vc)[0][:10])
    same_history(g, c)
    g.close()


@pytest.mark.parametrize("maxlen,chunk", [(3, None), (11, 256), (40, 4096)])
def test_per_txn_tiny_streams(gpu, maxlen, chunk):
    """Short keys ("" and < 8 bytes: the byte paths of the inline compare and
    copy), prefixes and \\x00 through the Python ConflictBatch mirror."""
    g = make_cs(chunk)
    for seed in range(3):
        g.load_history([], [], v0=0, oldest=0, removal_key=b"")
        c = CpuSpec()
        for batch, now, nold in tiny_stream(100 + seed, n_batches=12, max_txns=60, maxlen=maxlen, max_reads=3,
                                            max_writes=3):
            b = ConflictBatch(g)
            for snap, reads, writes in batch.txns():
                b.add_transaction(reads, writes, snap)
            v = b.detect_conflicts(now, nold)
            vc = c.detect_packed(batch, now, nold)
            assert np.array_equal(v, vc)
        same_history(g, c)
    g.close()


def test_per_txn_mixed_and_stream_growth(gpu):
    """Batches larger than the first staging allocation (the stream and the
    offset table grow mid-batch, after chunks were already sent)."""
    g = make_cs(1 << 12)
    c = CpuSpec()
    n = 120000
    big = [(b"k%030d" % i, b"k%030d\x00" % i) for i in range(n)]
    b = ConflictBatch(g)
    for i in range(0, n, 3):  # 40,000 transactions, ~9.5 MB of records (the first allocation is 4 MB)
        b.add_transaction([big[i]], [big[i + 1], big[i + 2]], 5)
    v = b.detect_conflicts(100, 0)
    from foundationdb_amd.batch import PackedBatch
    pb = PackedBatch.from_txns([(5, [big[i]], [big[i + 1], big[i + 2]]) for i in range(0, n, 3)])
    assert np.array_equal(v, c.detect_packed(pb, 100, 0))
    for batch, now, nold in mixed_stream(7, n_batches=8, max_txns=900, keyspace=3000):
        now += 100
        bb = ConflictBatch(g)
        for snap, reads, writes in batch.txns():
            bb.add_transaction(reads, writes, snap)
        assert np.array_equal(bb.detect_conflicts(now, nold), c.detect_packed(batch, now, nold))
    same_history(g, c)
    g.close()


def test_per_txn_errors(gpu):
    """A bad range (begin >= end) or an over-long key fails
    its addTransaction (FDBCS_E_RANGE / FDBCS_E_KEY); that transaction is not
    added and the batch and the history go on unchanged."""
    from foundationdb_amd.batch import PackedBatch
    g = ConflictSet()
    c = CpuSpec()
    b = ConflictBatch(g)
    b.add_transaction([(b"a", b"b")], [(b"a", b"c")], 1)
    with pytest.raises(FdbcsError) as e:
        b.add_transaction([(b"b", b"b")], [], 1)  # empty read range
    assert e.value.status == _abi.E_RANGE
    with pytest.raises(FdbcsError) as e:
        b.add_transaction([(b"c", b"d")], [(b"z", b"y")], 1)  # a good read, then a reversed write
    assert e.value.status == _abi.E_RANGE
    with pytest.raises(FdbcsError) as e:
        b.add_transaction([(b"a", b"b" * (_abi.MAX_KEY + 1))], [], 1)
    assert e.value.status == _abi.E_KEY
    b.add_transaction([], [(b"c", b"d")], 1)
    assert g._lib.fdbcs_batch_txn_count(g.handle) == 2
    v = b.detect_conflicts(10, 0)
    pb = PackedBatch.from_txns([(1, [(b"a", b"b")], [(b"a", b"c")]), (1, [], [(b"c", b"d")])])
    assert np.array_equal(v, c.detect_packed(pb, 10, 0))
    same_history(g, c)
    g.close()


def ConflictBatch_run(g, txns, now, nold):
    b = ConflictBatch(g)
    for snap, reads, writes in txns:
        b.add_transaction(reads, writes, snap)
    return b.detect_conflicts(now, nold)


def test_detect_without_batch_is_state_error(gpu):
    g = ConflictSet()
    assert g._lib.fdbcs_batch_detect(g.handle, 20, 0, None) == _abi.E_STATE  # no ConflictBatch open
    g.close()
