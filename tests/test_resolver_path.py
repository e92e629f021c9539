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


# ---- borrowed batches (fdbcs_config.flags FDBCS_BORROW_*: the adds record the
# caller's range arrays only; detectConflicts checks and packs them on host
# threads -- SkipList.cpp:993-1004 borrows the keys the same way) ----

BORROW_ALWAYS, BORROW_LARGE = 1, 2


@pytest.mark.parametrize("maxlen", [3, 40])
def test_borrowed_tiny_and_mixed_streams(gpu, maxlen):
    """Borrowed batches (every one, FDBCS_BORROW_ALWAYS) through the Python
    ConflictBatch mirror: "" and short keys, prefixes, \\x00, long keys, empty
    transactions, then larger mixed batches -- verdicts and the whole history as
    the oracle's after every batch."""
    g = ConflictSet(flags=BORROW_ALWAYS)
    c = CpuSpec()
    for batch, now, nold in tiny_stream(300 + maxlen, n_batches=12, max_txns=60, maxlen=maxlen, max_reads=3,
                                        max_writes=3):
        v = ConflictBatch_run(g, batch.txns(), now, nold)
        assert np.array_equal(v, c.detect_packed(batch, now, nold))
        same_history(g, c)
    for batch, now, nold in mixed_stream(11, n_batches=6, max_txns=9000, keyspace=40000):
        now += 2000
        v = ConflictBatch_run(g, batch.txns(), now, nold)
        assert np.array_equal(v, c.detect_packed(batch, now, nold))
    same_history(g, c)
    g.close()


def _long_key_stream(seed, n_batches, T):
    """Batches of short and long (> 17 bytes, tails) keys over a small key
    space, so reads hit the previous batches' writes."""
    import random
    rng = random.Random(seed)
    now = 1000

    def key(i):
        return (b"tenant/%03d/" % (i % 7)) * 3 + b"%05d" % i if i % 3 == 0 else b"k%05d" % i

    for _ in range(n_batches):
        now += rng.randint(20, 60)
        txns = []
        for _t in range(T):
            def rr():
                a = rng.randrange(6000)
                k = key(a)
                return (k, k + b"\x00") if rng.random() < 0.6 else tuple(sorted((k, key(a + rng.randint(1, 40)))))
            rs = [r for r in (rr() for _ in range(rng.randint(0, 3))) if r[0] < r[1]]
            ws = [r for r in (rr() for _ in range(rng.randint(0, 2))) if r[0] < r[1]]
            txns.append((now - rng.randint(1, 120), rs, ws))
        yield txns, now, now - rng.randint(150, 400)


def test_borrowed_back_to_back_long_keys(gpu):
    """Back-to-back borrowed batches with short and long keys (tails: the
    merge of one batch still reads its batch's tails while the host packs the
    next), verdicts as the oracle's every batch, the history at a midpoint
    (a dump queues work on the stream between batches) and at the end."""
    from foundationdb_amd.batch import PackedBatch
    g = ConflictSet(flags=BORROW_ALWAYS)
    c = CpuSpec()
    for i, (txns, now, nold) in enumerate(_long_key_stream(17, 14, 2500)):
        v = ConflictBatch_run(g, txns, now, nold)
        assert np.array_equal(v, c.detect_packed(PackedBatch.from_txns(txns), now, nold)), i
        if i == 8:
            same_history(g, c)
    same_history(g, c)
    g.close()


def test_borrowed_budget_refresh_under_pressure(gpu):
    """The budget refresh (engine.hip refresh_state) adopts the mirror slot of
    the batch before the last one while the last one's update still runs.
    With a small tail arena and an empty initial pool, refreshes, pool growth
    and tail-arena growth come every few batches: verdicts as the oracle's
    every batch and the history at the end."""
    from foundationdb_amd.batch import PackedBatch
    g = ConflictSet(flags=BORROW_ALWAYS, tail_arena_bytes=1 << 16)
    c = CpuSpec()
    for i, (txns, now, nold) in enumerate(_long_key_stream(23, 24, 1500)):
        v = ConflictBatch_run(g, txns, now, nold)
        assert np.array_equal(v, c.detect_packed(PackedBatch.from_txns(txns), now, nold)), i
    same_history(g, c)
    g.close()


def _ranges(lib_keys, spec):
    """ctypes Range array over the bytes of lib_keys (a bytearray the test keeps
    and later overwrites): spec = [(begin offset, begin len, end offset, end len)]."""
    import ctypes as C
    arr = (_abi.Range * max(1, len(spec)))()
    base = C.addressof((C.c_char * len(lib_keys)).from_buffer(lib_keys))
    for i, (bo, bl, eo, el) in enumerate(spec):
        arr[i].begin, arr[i].begin_len, arr[i].end, arr[i].end_len = base + bo, bl, base + eo, el
    return arr


def test_borrowed_keys_overwritten_after_detect(gpu):
    """a borrowed batch whose keys (and range arrays) the
    caller overwrites right after detectConflicts returns -- nothing of the
    library may still read them.  Each batch's buffers are scribbled over
    before the next batch; the history must equal the oracle's."""
    import random
    from foundationdb_amd.batch import PackedBatch
    g = ConflictSet(flags=BORROW_ALWAYS)
    c = CpuSpec()
    lib = g._lib
    rng = random.Random(5)
    now = 100
    for _ in range(6):
        now += 50
        txns = []
        for _t in range(3000):
            def rr():
                a = rng.randrange(5000)
                k = b"key%06d" % a
                return (k, k + b"\x00") if rng.random() < 0.7 else (k, b"key%06d" % (a + rng.randint(1, 30)))
            txns.append((now - rng.randint(1, 40), [rr() for _ in range(rng.randint(0, 3))],
                         [rr() for _ in range(rng.randint(0, 2))]))
        buf = bytearray()
        specs = []
        for snap, reads, writes in txns:
            sp = []
            for b, e in list(reads) + list(writes):
                bo = len(buf); buf += b
                eo = len(buf); buf += e
                sp.append((bo, len(b), eo, len(e)))
            specs.append((snap, sp, len(reads)))
        arrays = []
        assert lib.fdbcs_batch_begin(g.handle) == 0
        for snap, sp, nr in specs:
            ra, wa = _ranges(buf, sp[:nr]), _ranges(buf, sp[nr:])
            arrays.append((ra, wa))
            assert lib.fdbcs_batch_add(g.handle, snap, ra, nr, wa, len(sp) - nr) == 0
        out = np.zeros(len(txns), np.uint8)
        assert lib.fdbcs_batch_detect(g.handle, now, now - 200, out.ctypes.data) == 0
        # the caller's arena is reused at once: keys and range arrays scribbled over
        buf[:] = bytes([0xA5]) * len(buf)
        for ra, wa in arrays:
            for a in (ra, wa):
                for x in a:
                    x.begin_len, x.end_len = 7, 3
        pb = PackedBatch.from_txns(txns)
        assert np.array_equal(out, c.detect_packed(pb, now, now - 200))
        same_history(g, c)
    g.close()


def test_borrowed_refusal(gpu):
    """A borrowed batch refuses nothing at add time: a range the add would
    refuse makes detectConflicts fail with that status (the reference ASSERTs
    inside detectConflicts, SkipList.cpp:1117/1127), names the transaction
    (fdbcs_batch_refused_txn), and leaves the history as it was; the next
    batch goes on."""
    g = ConflictSet(flags=BORROW_ALWAYS)
    c = CpuSpec()
    lib = g._lib
    good = [(1, [(b"a", b"b")], [(b"a", b"c")]), (1, [], [(b"c", b"d")])]
    for bad, code in (((1, [(b"b", b"b")], []), _abi.E_RANGE),
                      ((1, [(b"a", b"b" * (_abi.MAX_KEY + 1))], []), _abi.E_KEY)):
        before = g.dump_arrays()
        b = ConflictBatch(g)
        for snap, reads, writes in good[:1] + [bad] + good[1:]:
            b.add_transaction(reads, writes, snap)  # (no refusal here)
        with pytest.raises(FdbcsError) as e:
            b.detect_conflicts(10, 0)
        assert e.value.status == code
        assert lib.fdbcs_batch_refused_txn(g.handle) == 1
        after = g.dump_arrays()
        assert all(np.array_equal(x, y) for x, y in zip(before, after))
    from foundationdb_amd.batch import PackedBatch
    v = ConflictBatch_run(g, good, 10, 0)
    assert lib.fdbcs_batch_refused_txn(g.handle) == -1
    assert np.array_equal(v, c.detect_packed(PackedBatch.from_txns(good), 10, 0))
    same_history(g, c)
    g.close()


def test_borrowed_first_batch_past_the_initial_offsets(gpu):
    """A conflict set whose very first per-transaction batch is borrowed and
    larger than the stage's initial offset table (8,192 entries): the table
    grows at detect without copying entries the adds never wrote (a 10^6-txn
    first batch read past the old table: bench.py --config 5 --borrow always
    crashed)."""
    g = ConflictSet(flags=BORROW_ALWAYS)
    c = CpuSpec()
    wl = Workload(2, txns=200_000)
    run = wl.prepare_run(0, 2)
    us, add_us, verdicts = run.run(g)
    for i in range(2):
        b, now, nold = wl.batch(i)
        assert np.array_equal(verdicts[i], c.detect_packed(b, now, nold)), i
    same_history(g, c)
    g.close()


def test_borrowed_large_batches_match_oracle(gpu):
    """Config 5's shape through the bench's native Resolver loop with
    FDBCS_BORROW_LARGE: the first 10^6-transaction batch copies its keys
    (no earlier batch), the next ones borrow and pack on host threads in
    rounds whose copies overlap the packing -- verdicts and history as the
    oracle's."""
    g = ConflictSet(flags=BORROW_LARGE)
    c = CpuSpec()
    wl = Workload(5, txns=1_000_000)
    nb = 3
    run = wl.prepare_run(0, nb)
    us, add_us, verdicts = run.run(g)
    for i in range(nb):
        b, now, nold = wl.batch(i)
        vc = c.detect_packed(b, now, nold)
        assert np.array_equal(verdicts[i], vc), (i, np.nonzero(verdicts[i] != vc)[0][:10])
    same_history(g, c)
    assert add_us[1] < 0.6 * add_us[0], add_us  # (borrowed adds record pointers only)
    g.close()


@pytest.mark.parametrize("live", [False, True])
@pytest.mark.parametrize("cfg,T,nb", [(2, 5000, 30), (3, 3000, 12), (4, 800, 8)])
def test_borrowed_helpers_resolver_loop(gpu, cfg, T, nb, live, monkeypatch):
    """Borrowed batches in the steady state: the adds record pointers and
    helper threads check and pack chunks of 64 transactions into the stream
    while the adds go on (stage.hip lb_work), copying the finished prefix to
    the device (default) or publishing it to the live kernel
    (FDBCS_BORROW_LIVE=1).  The bench's native Resolver loop against the
    oracle; with live=True most batches must have gone live."""
    monkeypatch.setenv("FDBCS_BORROW_LIVE", "1" if live else "0")
    g = ConflictSet(flags=BORROW_ALWAYS)
    c = CpuSpec()
    wl = Workload(cfg, txns=T)
    run = wl.prepare_run(0, nb)
    s0 = g.batch_stats()
    us, add_us, verdicts = run.run(g)
    s1 = g.batch_stats()
    for i in range(nb):
        b, now, nold = wl.batch(i)
        vc = c.detect_packed(b, now, nold)
        assert np.array_equal(verdicts[i], vc), (i, np.nonzero(verdicts[i] != vc)[0][:10])
    same_history(g, c)
    if live:
        assert s1["live_batches"] - s0["live_batches"] >= nb - 3, (s0, s1)
    else:
        assert s1["live_batches"] == s0["live_batches"], (s0, s1)
    g.close()


@pytest.mark.parametrize("live", [False, True])
def test_borrowed_helpers_fallbacks(gpu, live, monkeypatch):
    """Borrowed batches whose helpers run past their capacities -- twice the
    transactions, then the same count with 150-byte keys (key bytes past the
    cap), then a refused transaction in the middle of a live batch -- fall
    back to the whole-batch ingest (or refuse the batch) and stay exact."""
    from foundationdb_amd.batch import PackedBatch
    import random
    monkeypatch.setenv("FDBCS_BORROW_LIVE", "1" if live else "0")
    g = ConflictSet(flags=BORROW_ALWAYS)
    c = CpuSpec()
    rng = random.Random(9)
    now = 1000

    def batch(n, klen):
        txns = []
        for _ in range(n):
            def rr():
                a = rng.randrange(20000)
                k = (b"%08d" % a) * (klen // 8 + 1)
                k = k[:klen]
                return (k, k + b"\x00")
            txns.append((now - rng.randint(1, 50), [rr() for _ in range(2)], [rr()]))
        return txns

    shapes = [(1000, 16)] * 4 + [(2000, 16), (2000, 16), (2000, 150), (2000, 16), (2000, 16)]
    for n, klen in shapes:
        now += 100
        txns = batch(n, klen)
        v = ConflictBatch_run(g, txns, now, now - 400)
        assert np.array_equal(v, c.detect_packed(PackedBatch.from_txns(txns), now, now - 400))
        same_history(g, c)
    # a refused transaction deep in a live batch: the batch fails, nothing changes, the next one is exact
    before = g.dump_arrays()
    now += 100
    txns = batch(2000, 16)
    b = ConflictBatch(g)
    for i, (snap, reads, writes) in enumerate(txns):
        b.add_transaction(reads if i != 1500 else [(b"zz", b"aa")], writes, snap)
    with pytest.raises(FdbcsError) as e:
        b.detect_conflicts(now, now - 400)
    assert e.value.status == _abi.E_RANGE
    assert g._lib.fdbcs_batch_refused_txn(g.handle) == 1500
    assert all(np.array_equal(x, y) for x, y in zip(before, g.dump_arrays()))
    for _ in range(3):
        now += 100
        txns = batch(2000, 16)
        v = ConflictBatch_run(g, txns, now, now - 400)
        assert np.array_equal(v, c.detect_packed(PackedBatch.from_txns(txns), now, now - 400))
    same_history(g, c)
    g.close()
