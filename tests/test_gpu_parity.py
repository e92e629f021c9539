"""GPU parity: the HIP engine vs the CPU oracle, bit-exact on verdicts and history.

Every comparison checks the verdict bytes, the full post-batch boundary list
(keys and versions), removalKey, oldestVersion and the header version
(SURVEY.md §8c).  Oracle: oracle/cpu_spec.cpp (itself checked against the
pure-Python spec and the golden fixtures in test_oracle.py).
"""
import json
import os

import numpy as np
import pytest

from foundationdb_amd import ConflictBatch, ConflictSet, FdbcsError
from foundationdb_amd import _abi
from foundationdb_amd.batch import PackedBatch
from foundationdb_amd.workload import Workload
from gen import mixed_stream, tiny_stream
from oracle import CpuSpec, SpecBatch, SpecConflictSet

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def same_history(g, c):
    gv, gl, go, gk = g.dump_arrays()
    cv, cl, co, ck = c.dump_arrays()
    assert len(gv) == len(cv), (len(gv), len(cv))
    if len(gv) == 0:
        return
    assert np.array_equal(gv, cv), "versions differ"
    assert np.array_equal(gl, cl), "key lengths differ"
    n = int(gl.astype(np.int64).sum())
    assert np.array_equal(gk[:n], ck[:n]), "key bytes differ"


def check_pair(g, c, batch, now, nold, history=True):
    vg = g.detect_packed(batch, now, nold)
    vc = c.detect_packed(batch, now, nold)
    assert np.array_equal(vg, vc), (np.nonzero(vg != vc)[0][:10], vg[:20], vc[:20])
    assert g.oldest_version == c.oldest_version
    if history:
        same_history(g, c)
        assert g.removal_key() == c.removal_key()
    return vg


@pytest.fixture(scope="module")
def cs(gpu):
    g = ConflictSet()
    yield g
    g.close()


def test_golden_fixtures(cs):
    for name in ["tiny_alphabet", "long_keys", "clear_mid_stream", "appendix_c"]:
        with open(os.path.join(GOLDEN, f"{name}.json")) as f:
            streams = json.load(f)["streams"]
        for stream in streams:
            cs.clear(0)
            cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
            for e in stream:
                if "clear_before" in e:
                    cs.clear(e["clear_before"])
                txns = [(s, [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in r],
                         [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in w]) for s, r, w in e["txns"]]
                v = cs.detect_packed(PackedBatch.from_txns(txns), e["now"], e["new_oldest"])
                assert list(v) == e["verdict"], name
                assert [[k.hex(), ver] for k, ver in cs.history()] == e["history"], name
                assert cs.removal_key().hex() == e["removal_key"], name
                assert cs.oldest_version == e["oldest"]
                assert cs.header_version == e["v0"]


@pytest.mark.parametrize("maxlen", [3, 11, 40])
def test_tiny_streams(cs, maxlen):
    for seed in range(25):
        cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
        c = CpuSpec()
        for batch, now, nold in tiny_stream(seed * 13 + maxlen, n_batches=30, maxlen=maxlen):
            check_pair(cs, c, batch, now, nold)


def test_mixed_streams(cs):
    for seed in range(4):
        cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
        c = CpuSpec()
        for batch, now, nold in mixed_stream(seed, n_batches=15, max_txns=600, keyspace=5000):
            check_pair(cs, c, batch, now, nold)


def test_per_transaction_api_appends(cs):
    """ConflictBatch mirror: addTransaction x T + detectConflicts appends like the reference."""
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    spec = SpecConflictSet()
    rounds = [
        (10, 0, [([], [(b"a", b"b")], 0)]),
        (20, 5, [([(b"a", b"b")], [], 1), ([(b"a", b"b")], [(b"a", b"c")], 10), ([], [(b"c", b"d")], 1),
                 ([(b"b", b"bb")], [], 15)]),
    ]
    for now, nold, txns in rounds:
        b = ConflictBatch(cs)
        sb = SpecBatch(spec)
        for r, w, s in txns:
            b.add_transaction(r, w, s)
            sb.add_transaction(r, w, s)
        nc, to = [99], [98]
        b.detect_conflicts(now, nold, nc, to)
        v, snc, sto = sb.detect_conflicts(now, nold)
        assert nc == [99] + snc and to == [98] + sto
    assert cs.history() == spec.history()


def test_per_transaction_skip_runs(cs):
    """fdbcs_batch_skip: runs of range-less transactions in one call (how a
    protocol-B shard receives the transactions the proxy did not send it)
    give the verdicts and history of adding them one by one."""
    import random
    for seed in range(3):
        cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
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
            b = ConflictBatch(cs)
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
            v = b.detect_conflicts(now, nold)
            assert np.array_equal(v, vc)
        assert cs.history() == c.history()
    b = ConflictBatch(cs)  # a batch of nothing but skipped transactions
    b.skip(7)
    assert b.detect_conflicts(10 ** 9, 0).tolist() == [2] * 7


def test_per_transaction_chunk_edges(gpu, monkeypatch):
    """The staging's chunk copies at every position: 4 KiB chunks and an early
    last chunk 4 KiB before where the previous batch's stream ended
    (FDBCS_STAGE_CHUNK / FDBCS_STAGE_EARLY, read when the conflict set is
    made), over batches whose sizes jump up and down -- so the early chunk
    falls inside, at the end of and past the next batch's stream."""
    import random
    monkeypatch.setenv("FDBCS_STAGE_CHUNK", "4096")
    monkeypatch.setenv("FDBCS_STAGE_EARLY", "4096")
    g = ConflictSet()
    try:
        rng = random.Random(5)
        c = CpuSpec()
        sizes = [300, 20, 0, 500, 450, 5, 260, 1, 600]
        now = 1000
        for i, T in enumerate(sizes):
            now += rng.randint(50, 200)
            nold = max(0, now - 600)
            batch = next(mixed_stream(i, n_batches=1, max_txns=max(T, 1), keyspace=2000))[0]
            txns = [(min(snap, now - 1), r, w) for snap, r, w in list(batch.txns())[:T]]
            vc = c.detect_packed(PackedBatch.from_txns(txns), now, nold)
            b = ConflictBatch(g)
            for snap, r, w in txns:
                b.add_transaction(r, w, snap)
            v = b.detect_conflicts(now, nold)
            assert np.array_equal(v, vc), i
            assert g.history() == c.history(), i
    finally:
        g.close()


@pytest.mark.parametrize("cfg,T,nb", [(1, 2500, 20), (2, 800, 25), (3, 800, 25), (4, 400, 12)])
def test_workload_configs_small(cs, cfg, T, nb):
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    c = CpuSpec()
    wl = Workload(cfg, txns=T)
    for i in range(nb):
        batch, now, nold = wl.batch(i)
        check_pair(cs, c, batch, now, nold, history=(i % 5 == 4 or i == nb - 1))


def test_sort_splitters_outlive_their_keys(cs):
    """Splitters are the previous batch's quantiles; with long keys sharing
    their first 17 bytes (config 4) comparing against them needs their tails,
    which must not be read from the current batch's key slots (a smaller
    batch does not even have those slots)."""
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    c = CpuSpec()
    big, small = Workload(4, txns=1200), Workload(4, txns=90)
    for i in range(10):
        batch, now, nold = (big if i % 2 == 0 else small).batch(i)
        check_pair(cs, c, batch, now, nold, history=(i % 3 == 2 or i == 9))


@pytest.mark.parametrize("buckets", ["1", "2", "8"])
def test_sort_bucket_paths(cs, buckets):
    """Few sample-sort buckets push them past the register path (128 records)
    onto the LDS path (<= 512) and the global-memory ranking path; results
    must not change.  Also exercises the re-sample after an unbalanced batch."""
    os.environ["FDBCS_TEST_SORT_BUCKETS"] = buckets
    try:
        cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
        c = CpuSpec()
        wl = Workload(3, txns=300)
        for i in range(4):
            b, now, nold = wl.batch(i)
            check_pair(cs, c, b, now, nold)
    finally:
        del os.environ["FDBCS_TEST_SORT_BUCKETS"]


def test_key_range_resolvers_on_gpu(gpu):
    """Three key-range resolvers (three conflict sets on one GPU) fed by the
    native proxy split; the GPU verdict scatter + MIN combine and every
    resolver's history must equal three oracle resolvers'."""
    import torch
    from foundationdb_amd.resolvers import KeyRangeResolvers, combine, scatter_verdicts, uniform_bounds

    kr = KeyRangeResolvers(uniform_bounds(3))
    gres = [ConflictSet() for _ in range(3)]
    cres = [CpuSpec() for _ in range(3)]
    wl = Workload(2, txns=1500)
    try:
        for i in range(8):
            batch, now, nold = wl.batch(i)
            full = torch.full((batch.T,), 2, dtype=torch.uint8, device="cuda")
            parts = []
            for g in range(3):
                sub, idx = kr.split(batch, g)
                vg = gres[g].detect_packed(sub, now, nold)
                vc = cres[g].detect_packed(sub, now, nold)
                assert np.array_equal(vg, vc), (i, g)
                part = torch.full((batch.T,), 2, dtype=torch.uint8, device="cuda")
                dv = torch.from_numpy(vg.copy()).cuda()
                di = torch.from_numpy(idx).cuda()
                torch.cuda.synchronize()
                scatter_verdicts(None, dv.data_ptr(), di.data_ptr(), len(idx), part.data_ptr())
                full = torch.minimum(full, part)
                parts.append((vc, idx))
            torch.cuda.synchronize()
            assert np.array_equal(full.cpu().numpy(), combine(batch.T, parts))
        for g in range(3):
            same_history(gres[g], cres[g])
    finally:
        for x in gres:
            x.close()


def test_config2_full_batches(cs):
    """Config 2 at its real batch size (5,000 txns, 5R+2W) from an empty history."""
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    c = CpuSpec()
    wl = Workload(2)
    for i in range(30):
        batch, now, nold = wl.batch(i)
        check_pair(cs, c, batch, now, nold, history=(i % 10 == 9))


def test_steady_state_preloaded_history(cs):
    """A multi-million-boundary history with old and new versions; compaction active."""
    rng = np.random.default_rng(5)
    n = 1_500_000
    raw = np.unique(rng.integers(0, 2**63, size=n, dtype=np.int64))
    keys = raw.astype(">u8").view(np.uint8).reshape(-1, 8)
    blob = np.concatenate([keys, np.zeros((len(raw), 8), np.uint8)], axis=1).reshape(-1).copy()  # 16-byte keys
    lens = np.full(len(raw), 16, np.uint32)
    offs = (np.arange(len(raw), dtype=np.uint64) * 16)
    vers = rng.integers(4_000_000, 10_000_000, size=len(raw)).astype(np.int64)
    c = CpuSpec()
    cs.load_history_arrays(len(raw), vers, lens, offs, blob, v0=0, oldest=4_000_000, removal_key=b"")
    c.load_history_arrays(len(raw), vers, lens, offs, blob, v0=0, oldest=4_000_000, removal_key=b"")
    same_history(cs, c)
    wl = Workload(2)
    for i in range(12):
        batch, now, nold = wl.batch(i)
        check_pair(cs, c, batch, now, nold, history=(i in (0, 11)))


def test_config2_steady_state_independent(cs):
    """Config 2 past its 5 M-version window: 540 batches of 5,000 transactions
    (compaction from batch ~500 on, H ~ 10 M boundaries; ~80 s of oracle).  The GPU builds its
    history through the pipelined whole-batch prefill (the bench's), the CPU
    oracle independently from the same generated batches -- not from the GPU's
    dump -- and the two histories must be identical; then 8 more batches
    through the checked path compare verdicts and history."""
    import ctypes as C
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    c = CpuSpec()
    wl = Workload(2)
    n = 540
    wl.prefill(cs, 0, n)
    out = np.zeros(8192, np.uint8)
    for i in range(n):
        v, now, nold = wl.view(i)
        assert v.txn_count <= len(out)
        assert c._l.orc_detect(c._h, C.byref(v), now, nold, out.ctypes.data) == 0
    assert cs.history_size() > 5_000_000
    same_history(cs, c)
    assert cs.removal_key() == c.removal_key()
    for i in range(n, n + 8):
        batch, now, nold = wl.batch(i)
        check_pair(cs, c, batch, now, nold, history=(i == n + 7))


def test_wide_reads_three_level_range_max(cs):
    """Reads spanning up to the whole history (> 3 x 4096 directory entries):
    the read check's entry / 64-group / 4096-group maxima.  Low versions
    everywhere except a few spikes, so each verdict hinges on whether a spike
    lies inside the read -- at any level of the range maximum."""
    rng = np.random.default_rng(11)
    n = 2_600_000
    raw = np.unique(rng.integers(0, 2**63, size=n, dtype=np.int64))
    n = len(raw)
    keys = raw.astype(">u8").view(np.uint8).reshape(-1, 8)
    blob = np.concatenate([keys, np.zeros((n, 8), np.uint8)], axis=1).reshape(-1).copy()
    lens = np.full(n, 16, np.uint32)
    offs = np.arange(n, dtype=np.uint64) * 16
    vers = rng.integers(100, 1000, size=n).astype(np.int64)
    spikes = rng.choice(n, size=4, replace=False)
    vers[spikes] = 10_000
    c = CpuSpec()
    cs.load_history_arrays(n, vers, lens, offs, blob, v0=0, oldest=0, removal_key=b"")
    c.load_history_arrays(n, vers, lens, offs, blob, v0=0, oldest=0, removal_key=b"")
    key = lambda i: bytes(blob[16 * i:16 * i + 16])
    txns = []
    for t in range(3000):
        span = int(n * 10 ** rng.uniform(-4, 0))
        a = int(rng.integers(0, max(1, n - span)))
        b = min(n - 1, a + max(1, span))
        if t % 7 == 0:
            a, b = 0, n - 1
        txns.append((int(rng.choice([500, 5_000, 20_000])), [(key(a), key(b))], []))
    batch = PackedBatch.from_txns(txns)
    vg = cs.detect_packed(batch, 30_000, 0)
    vc = c.detect_packed(batch, 30_000, 0)
    assert np.array_equal(vg, vc)
    assert 0 < int((vg == _abi.CONFLICT).sum()) < len(txns)  # both outcomes occur


def test_empty_and_degenerate_batches(cs):
    cs.load_history([], [], v0=7, oldest=0, removal_key=b"")
    c = CpuSpec(v0=7)
    check_pair(cs, c, PackedBatch.from_txns([]), 10, 5)
    check_pair(cs, c, PackedBatch.from_txns([(1, [], [])] * 5), 11, 6)
    check_pair(cs, c, PackedBatch.from_txns([(1, [(b"a", b"b")], [])]), 12, 6)   # tooOld (oldest 6)
    check_pair(cs, c, PackedBatch.from_txns([(1, [], [(b"", b"\xff")])]), 13, 6)  # blind write commits
    check_pair(cs, c, PackedBatch.from_txns([(13, [(b"", b"\xff" * 30)], [(b"\x00", b"\x01")])]), 14, 7)


def test_errors_leave_state_intact(cs):
    cs.load_history([b"a", b"m"], [5, 6], v0=1, oldest=0, removal_key=b"")
    before = cs.history()
    with pytest.raises(FdbcsError) as ei:
        cs.detect_packed(PackedBatch.from_txns([(1, [(b"b", b"b")], [])]), 10, 0)
    assert ei.value.status == _abi.E_RANGE
    with pytest.raises(FdbcsError) as ei:
        cs.detect_packed(PackedBatch.from_txns([(1, [], [(b"z", b"a")])]), 10, 0)
    assert ei.value.status == _abi.E_RANGE
    with pytest.raises(FdbcsError) as ei:
        cs.detect_packed(PackedBatch.from_txns([(1, [], [(b"a", b"b" * 30002)])]), 10, 0)
    assert ei.value.status == _abi.E_KEY
    assert cs.history() == before


def test_load_dump_roundtrip(cs):
    keys = [b"", b"\x00", b"a", b"a\x00", b"ab" * 20, b"b", b"\xff" * 18]
    vers = [3, 1, 4, 1, 5, 9, 2]
    cs.load_history(keys, vers, v0=11, oldest=2, removal_key=b"ab" * 20)
    assert cs.history() == list(zip(keys, vers))
    assert cs.removal_key() == b"ab" * 20
    assert cs.header_version == 11 and cs.oldest_version == 2


@pytest.mark.parametrize("guard", ["1", None])
def test_sort_distribution_shift(cs, guard, monkeypatch):
    """The sort buckets by the previous batch's quantiles; a batch whose keys
    all lie outside them (a moved key distribution) overflows one bucket.
    With the guard (FDBCS_SORT_GUARD=1) it is re-bucketed by splitters from
    its own sample in the same batch (stats: sort_rebucketed).  By default the
    guard runs only after a batch whose largest bucket came near its staging
    row (engine.hip sort_guard): the first overflowed batch is then ranked by
    the bucket kernel's global path, and the next one, guarded, re-buckets.
    Verdicts and history must not change either way."""
    import random

    if guard:
        monkeypatch.setenv("FDBCS_SORT_GUARD", guard)
    else:
        monkeypatch.delenv("FDBCS_SORT_GUARD", raising=False)
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    c = CpuSpec()
    rng = random.Random(7)
    for i, prefix in enumerate([b"\x00", b"\x00", b"\xff", b"\x80", b"\x80"]):
        txns = []
        for _t in range(3000):
            k = prefix + rng.getrandbits(96).to_bytes(12, "big")
            w = prefix + rng.getrandbits(96).to_bytes(12, "big")
            txns.append((100 + 10 * i - rng.randint(1, 15), [(k, k + b"\x00")], [(w, w + b"\x00")]))
        check_pair(cs, c, PackedBatch.from_txns(txns), 100 + 10 * i, 90 + 10 * i)
        st = cs.batch_stats()
        if i in (2, 3):
            assert st["sort_rebucketed"] == (1 if guard or i == 3 else 0), st
        if i in (1, 4):
            assert st["sort_rebucketed"] == 0 and st["sort_max_bucket"] <= 512, st


@pytest.mark.parametrize("T,force", [(20000, None), (1500, "FDBCS_TEST_MULTIBLOCK_COMBINE"),
                                     (1500, "FDBCS_TEST_LARGE_BATCH"), (9000, None)])
def test_large_batches_multiblock_combine(cs, T, force):
    """Batches past one workgroup's register budget (2W > 32768 endpoints)
    combine with the multi-block kernels; large-batch mode (overlap edges and
    the grid decision) can be forced onto small ones."""
    if force:
        os.environ[force] = "1"
    try:
        cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
        c = CpuSpec()
        wl = Workload(2, txns=T)
        for i in range(6):
            batch, now, nold = wl.batch(i)
            check_pair(cs, c, batch, now, nold, history=(i % 2 == 1))
        wl3 = Workload(3, txns=T)  # Zipf: long intra-batch chains, touching ranges
        for i in range(6, 10):
            batch, now, nold = wl3.batch(i)
            check_pair(cs, c, batch, now, nold, history=(i % 2 == 1))
    finally:
        if force:
            os.environ.pop(force, None)


def test_zipf_full_batches_rounds(cs):
    """Config 3 at its full batch size (5,000 transactions, Zipf hot keys):
    the decision by rounds (k_decide_rounds, no overlap pairs) against the
    oracle, with the rounds it took in the batch stats."""
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    c = CpuSpec()
    wl = Workload(3, txns=5000)
    rounds = []
    for i in range(12):
        batch, now, nold = wl.batch(i)
        check_pair(cs, c, batch, now, nold, history=(i % 4 == 3))
        rounds.append(cs.batch_stats()["decision_rounds"])
    assert max(rounds) > 1, rounds  # (intra-batch conflicts did occur)


@pytest.mark.parametrize("lcap", ["0", "700"])
def test_rounds_items_past_lds(cs, lcap):
    """The rounds' item list (writes of U, candidate reads) partly or wholly in
    global memory instead of LDS (FDBCS_TEST_ROUNDS_LCAP)."""
    os.environ["FDBCS_TEST_ROUNDS_LCAP"] = lcap
    try:
        cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
        c = CpuSpec()
        wl = Workload(3, txns=2000)
        for i in range(5):
            batch, now, nold = wl.batch(i)
            check_pair(cs, c, batch, now, nold, history=(i == 4))
        same_history(cs, c)
        cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
        c = CpuSpec()
        for batch, now, nold in mixed_stream(11, n_batches=5, max_txns=500, keyspace=1500, wide=0.3):
            check_pair(cs, c, batch, now, nold, history=False)
        same_history(cs, c)
    finally:
        os.environ.pop("FDBCS_TEST_ROUNDS_LCAP", None)


def test_decision_long_chain(cs):
    """An alternating chain: t reads the key t-1 wrote and writes the next one,
    so t commits iff t-1 aborted -- every transaction flips the next, the
    worst case for the rounds (T + 1 of them)."""
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    c = CpuSpec()
    T = 700
    key = [b"chain%05d" % i for i in range(T + 1)]
    txns = [(5, [] if t == 0 else [(key[t], key[t] + b"\x00")], [(key[t + 1], key[t + 1] + b"\x00")])
            for t in range(T)]
    v = check_pair(cs, c, PackedBatch.from_txns(txns), 10, 0)
    assert list(v[:6]) == [2, 0, 2, 0, 2, 0]
    assert cs.batch_stats()["decision_rounds"] >= T // 2


def test_pipelined_submit_wait_matches_synchronous(cs):
    """fdbcs_batch_submit_packed / fdbcs_batch_wait (two batches in flight,
    overlapped host packing and H2D) give the synchronous path's verdicts and
    history; a synchronous call while batches are in flight is refused."""
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    c = CpuSpec()
    wl = Workload(2, txns=2000)
    batches = [wl.batch(i) for i in range(12)]
    got = []
    for i, (b, now, nold) in enumerate(batches):
        cs.submit_packed(b, now, nold)
        if i == 1:
            with pytest.raises(FdbcsError):
                cs.detect_packed(b, now, nold)
        if i >= 1:
            got.append(cs.wait())
    got.append(cs.wait())
    for (b, now, nold), vg in zip(batches, got):
        assert np.array_equal(vg, c.detect_packed(b, now, nold))
    same_history(cs, c)
    assert cs.removal_key() == c.removal_key()
