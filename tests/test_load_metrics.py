"""Resolver load metrics: iopsSample on the device.

CPU tests pin the sample structure: the reference's own known-answer test
(StorageMetrics.actor.h:81-93) and random differentials of getEstimate /
splitEstimate between libfdbcs.so's host sample and the oracle restatement
(oracle/load_sample.py).  GPU tests check the device roll of whole batches
(the Resolver.actor.cpp:146-151 loop) against the oracle, bit for bit: the
same sampled keys and amounts, the same queue, the same estimates and splits
after polls.
"""
import random

import numpy as np
import pytest

from foundationdb_amd import _abi
from foundationdb_amd.load_metrics import ALL_KEYS, KEY_BYTES_PER_SAMPLE, IopsSample
from foundationdb_amd.workload import Workload
from gen import mixed_stream, tiny_stream
from oracle.load_sample import SpecSample, key_between, roll_hash


def test_reference_known_answer_simple():
    """TEST_CASE("/fdbserver/StorageMetricSample/simple"), StorageMetrics.actor.h:81-93."""
    entries = [(b"Apple", 1000), (b"Banana", 2000), (b"Cat", 1000), (b"Cathode", 1000), (b"Dog", 1000)]
    for s in (IopsSample(1000), SpecSample(1000)):
        for k, m in entries:
            s.add_metric(k, m)
        assert s.get_estimate(b"A", b"D") == 5000
        assert s.get_estimate(b"A", b"E") == 6000
        assert s.get_estimate(b"B", b"C") == 2000


def test_key_between_follows_reference():
    """keyBetween (fdbclient/FDBTypes.h:304-325) cases."""
    assert key_between(b"abc", b"abd") == b"abd"
    assert key_between(b"ab", b"abcd") == b"abc"
    assert key_between(b"a", b"b") == b"b"
    assert key_between(b"", b"xyz") == b"x"
    assert key_between(b"abc", b"abc") == b"abc"
    assert key_between(b"x" * 6000, b"x" * 6001) == b"x" * 6001  # past SPLIT_KEY_SIZE_LIMIT


def test_roll_hash_vectors():
    """The draw function restated in numpy equals its definition on Python ints."""
    def mix(seed, seq, pos):
        M = 2**64 - 1
        z = (seed + seq * 0xD1B54A32D192ED03 + pos * 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    pos = np.arange(1000, dtype=np.uint64)
    h = roll_hash(12345, 7, pos)
    assert [int(x) for x in h[:50]] == [mix(12345, 7, int(p)) for p in pos[:50]]
    # the sampling probability is metric / units
    frac = float(np.mean((roll_hash(1, 2, np.arange(200000, dtype=np.uint64)) % np.uint64(20000)) < 116))
    assert abs(frac - 116 / 20000) < 0.0015


def _rand_entries(rng, n, alpha=b"ab\x00c", maxlen=4):
    out = []
    for _ in range(n):
        k = bytes(rng.choice(alpha) for _ in range(rng.randint(0, maxlen)))
        out.append((k, rng.choice([1, 5, 100, 1000, -1, 20000])))
    return out


@pytest.mark.parametrize("seed", range(6))
def test_sample_estimates_and_splits_match_oracle(seed):
    rng = random.Random(seed)
    g, o = IopsSample(1000), SpecSample(1000)
    for k, m in _rand_entries(rng, 300):
        if m < 0 and o.metric.get(k, 0) + m <= 0:
            continue  # keep metrics positive, as the Resolver's are
        g.add_metric(k, m)
        o.add_metric(k, m)
    assert g.items() == o.items()
    keys = [b"", b"a", b"ab", b"b", b"c", b"\x00", b"a\x00", b"ba", b"cc", b"\xff\xff"]
    for _ in range(200):
        b, e = sorted(rng.sample(keys, 2))
        assert g.get_estimate(b, e) == o.get_estimate(b, e)
        off = rng.randint(-500, o.get_estimate(b"", b"\xff\xff") + 500)
        for front in (True, False):
            assert g.split_estimate(b, e, off, front) == o.split_estimate(b, e, off, front), (b, e, off, front)


def test_empty_sample():
    g = IopsSample()
    assert g.get_estimate(*ALL_KEYS) == 0
    assert g.split_estimate(b"a", b"z", 100, True) == b"z"
    assert g.split_estimate(b"a", b"z", 100, False) == b"z"  # index() == end -> range.end (:41-42)
    assert g.size() == 0 and g.queue_size() == 0
    g.poll(1e9)


def test_add_batch_null_handle_is_arg_error():
    """fdbcs_sample_add_batch with no conflict set: FDBCS_E_ARG."""
    with pytest.raises(_abi.FdbcsError) as e:
        IopsSample().add_batch(_NoBatch(), 1.0)
    assert e.value.status == _abi.E_ARG


class _NoBatch:
    handle = None


@pytest.mark.gpu
def test_add_batch_without_resolved_batch_is_state_error(gpu):
    """fdbcs_sample_add_batch(cs, NULL) rolls the batch the conflict set last
    resolved through a host path; with none (a fresh set, or after a batch
    resolved on device memory) it is FDBCS_E_STATE (fdbcs.h)."""
    from foundationdb_amd import ConflictSet
    from foundationdb_amd.batch import DeviceBatch
    import torch

    cs = ConflictSet()
    with pytest.raises(_abi.FdbcsError) as e:
        IopsSample().add_batch(cs, 1.0)
    assert e.value.status == _abi.E_STATE
    wl = Workload(2, txns=200)
    b, now, nold = wl.batch(0)
    cs.detect_packed(b, now, nold)
    s = IopsSample()
    s.add_batch(cs, 1.0)  # the host batch is there
    v, now, nold = wl.view(1)
    db = DeviceBatch(v, torch.device("cuda", 0))
    out = torch.zeros(v.txn_count, dtype=torch.uint8, device="cuda")
    cs.detect_device(db.view, now, nold, out.data_ptr(), sync=True)
    with pytest.raises(_abi.FdbcsError) as e:
        s.add_batch(cs, 2.0)  # the last resolved batch came from device memory: nothing host-staged to roll
    assert e.value.status == _abi.E_STATE
    cs.close()


# ---------------------------------------------------------------- GPU

def _run_stream(cs, stream, units, seed, offset=100, poll_every=3):
    g, o = IopsSample(units, seed=seed), SpecSample(units, seed=seed)
    t = 0.0
    for i, (batch, now, nold) in enumerate(stream):
        cs.detect_packed(batch, now, nold)
        t += 0.4
        ng = g.add_batch(cs, t + 1.0, offset_per_key=offset)
        no = o.add_batch(batch, t + 1.0, offset_per_key=offset)
        assert ng == no, (i, ng, no)
        assert g.queue_size() == len(o.queue)
        if i % poll_every == 0:
            g.poll(t)
            o.poll(t)
        assert g.items() == o.items(), i
        assert g.get_estimate(*ALL_KEYS) == o.get_estimate(*ALL_KEYS)
    return g, o


@pytest.mark.gpu
def test_device_roll_tiny_streams(gpu):
    from foundationdb_amd import ConflictSet
    cs = ConflictSet(device=0)
    for seed in range(6):
        # units 110: keys of length >= 10 are added whole, shorter ones rolled
        g, o = _run_stream(cs, tiny_stream(seed, n_batches=12, maxlen=11), units=110, seed=seed)
        rng = random.Random(seed)
        keys = sorted({k for k, _ in o.items()} | {b"", b"a", b"b", b"c", b"\xff"})
        for _ in range(100):
            b, e = sorted(rng.sample(keys, 2))
            off = rng.randint(0, max(1, o.get_estimate(b, e)))
            for front in (True, False):
                assert g.split_estimate(b, e, off, front) == o.split_estimate(b, e, off, front)
    cs.close()


@pytest.mark.gpu
def test_device_roll_long_keys(gpu):
    """Begin keys of 0..300 B and up to 20 KB (metric >= units: added whole,
    no roll, StorageMetrics.actor.h:171-175), at the knobs' units."""
    from foundationdb_amd import ConflictSet
    from foundationdb_amd.batch import PackedBatch
    rng = random.Random(11)
    cs = ConflictSet(device=0)

    def key():
        r = rng.random()
        n = rng.randint(19890, 20010) if r < 0.02 else rng.randint(0, 300)
        return bytes(rng.randrange(256) for _ in range(n)) if n < 400 else bytes([rng.randrange(4)]) * n

    def rng_range():
        a = key()
        return (a, a + b"\x00")

    def stream():
        now = 100
        for _ in range(6):
            now += 10
            txns = [(now - 5, [rng_range() for _ in range(rng.randint(0, 3))],
                     [rng_range() for _ in range(rng.randint(0, 2))]) for _ in range(rng.randint(50, 400))]
            yield PackedBatch.from_txns(txns), now, now - 50

    g, o = _run_stream(cs, stream(), units=KEY_BYTES_PER_SAMPLE, seed=5, poll_every=2)
    assert any(len(k) >= 19900 and m >= KEY_BYTES_PER_SAMPLE for k, m in o.items())
    cs.close()


@pytest.mark.gpu
def test_device_roll_mixed_and_config2(gpu):
    from foundationdb_amd import ConflictSet
    from foundationdb_amd.workload import Workload
    cs = ConflictSet(device=0)
    _run_stream(cs, mixed_stream(3, n_batches=8, max_txns=600), units=2000, seed=99)
    wl = Workload(2, txns=5000)
    stream = (wl.batch(i) for i in range(6))
    g, o = _run_stream(cs, stream, units=KEY_BYTES_PER_SAMPLE, seed=7, poll_every=2)
    assert g.size() > 0
    # the master's balancing queries (masterserver.actor.cpp:964-1020)
    total = g.get_estimate(*ALL_KEYS)
    for front in (True, False):
        key, used = g.resolution_split(b"", b"\xff\xff", total // 3, front)
        assert key == o.split_estimate(b"", b"\xff\xff", total // 3, front)
        assert used == (o.get_estimate(b"", key) if front else o.get_estimate(key, b"\xff\xff"))
    # everything expires
    g.poll(1e9)
    o.poll(1e9)
    assert g.size() == 0 and g.get_estimate(*ALL_KEYS) == 0 and o.items() == []
    cs.close()


@pytest.mark.gpu
def test_key_range_resolvers_sample_their_sub_batches(gpu):
    """resolverCount > 1 (Resolver.actor.cpp:146): three key-range resolvers,
    each sampling the sub-batch the proxy split sends it; the master's
    ResolutionMetricsRequest / ResolutionSplitRequest answers
    (masterserver.actor.cpp:964-1020) equal three oracle samples'."""
    from foundationdb_amd import ConflictSet
    from foundationdb_amd.resolvers import KeyRangeResolvers, uniform_bounds
    from foundationdb_amd.workload import Workload

    kr = KeyRangeResolvers(uniform_bounds(3))
    lo_hi = [(b"", kr.bounds[0]), (kr.bounds[0], kr.bounds[1]), (kr.bounds[1], b"\xff\xff")]
    gres = [ConflictSet(device=0) for _ in range(3)]
    gs = [IopsSample(KEY_BYTES_PER_SAMPLE, seed=g) for g in range(3)]
    os_ = [SpecSample(KEY_BYTES_PER_SAMPLE, seed=g) for g in range(3)]
    wl = Workload(2, txns=3000)
    t = 0.0
    for i in range(8):
        batch, now, nold = wl.batch(i)
        t += 0.3
        for g in range(3):
            sub, _idx = kr.split(batch, g)
            gres[g].detect_packed(sub, now, nold)
            assert gs[g].add_batch(gres[g], t + 1.0) == os_[g].add_batch(sub, t + 1.0)
            gs[g].poll(t)
            os_[g].poll(t)
    metrics = [s.get_estimate(*ALL_KEYS) for s in gs]
    assert metrics == [o.get_estimate(*ALL_KEYS) for o in os_]
    src = int(np.argmax(metrics))
    amount = max(1, (metrics[src] - min(metrics)) // 2)
    b, e = lo_hi[src]
    for front in (True, False):
        key, used = gs[src].resolution_split(b, e, amount, front)
        assert key == os_[src].split_estimate(b, e, amount, front)
        assert b <= key <= e
        assert used == (os_[src].get_estimate(b, key) if front else os_[src].get_estimate(key, e))
    for x in gres:
        x.close()


@pytest.mark.gpu
def test_device_roll_explicit_device_batch(gpu):
    """fdbcs_sample_add_batch over a caller-owned device batch view (the
    fdbcs_detect_device path); a pipelined submit leaves no 'last batch'."""
    import torch
    from foundationdb_amd import ConflictSet
    from foundationdb_amd._abi import BatchView
    from foundationdb_amd.workload import Workload

    cs = ConflictSet(device=0)
    wl = Workload(2, txns=2000)
    g, o = IopsSample(2000, seed=3), SpecSample(2000, seed=3)
    for i in range(4):
        b, _now, _nold = wl.batch(i)
        bufs = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in
                (b.snapshot, b.read_off, b.write_off, b.key_off.view(np.int64), b.key_len.view(np.int32),
                 b.key_bytes)]
        torch.cuda.synchronize()
        dv = BatchView()
        dv.txn_count, dv.read_count, dv.write_count = b.T, b.R, b.W
        dv.snapshot, dv.read_off, dv.write_off = bufs[0].data_ptr(), bufs[1].data_ptr(), bufs[2].data_ptr()
        dv.key_off, dv.key_len, dv.key_bytes = bufs[3].data_ptr(), bufs[4].data_ptr(), bufs[5].data_ptr()
        dv.key_bytes_len = int(b.key_bytes.size)
        assert g.add_batch(cs, 1.0 + i, dev_batch=dv) == o.add_batch(b, 1.0 + i)
        assert g.items() == o.items()
    b, now, nold = wl.batch(10)
    cs.submit_packed(b, now, nold)
    cs.wait()
    with pytest.raises(_abi.FdbcsError):
        g.add_batch(cs, 9.0)
    cs.close()


def _detect_txns(cs, batch, now, nold):
    """The Resolver's per-transaction calls (ConflictBatch, addTransaction x T, detectConflicts)."""
    from foundationdb_amd.conflict_set import ConflictBatch
    cb = ConflictBatch(cs)
    for snap, reads, writes in batch.txns():
        cb.add_transaction(reads, writes, snap)
    return cb.detect_conflicts(now, nold)


@pytest.mark.gpu
def test_attached_roll_in_the_ingest(gpu):
    """fdbcs_sample_attach: the per-transaction ingest rolls every range for
    the attached sample (ADVICE/VERDICT r03: the roll no longer queues behind
    the history update and synchronizes); add_batch then only inserts.  Same
    keys, amounts, queue, estimates and splits as the oracle after every
    batch -- including batches the caller does not add (their draws are
    unused), packed batches and a different offset in between (the
    synchronous roll), re-attachment, and a conflict set destroyed before its
    sample."""
    from foundationdb_amd import ConflictSet
    cs = ConflictSet(device=0)
    for units, stream in ((110, list(tiny_stream(5, n_batches=14, maxlen=11))),
                          (KEY_BYTES_PER_SAMPLE, [Workload(2, txns=5000).batch(i) for i in range(6)])):
        g, o = IopsSample(units, seed=21), SpecSample(units, seed=21)
        g.attach(cs)
        t = 0.0
        for i, (batch, now, nold) in enumerate(stream):
            packed = i % 5 == 3
            if packed:
                cs.detect_packed(batch, now, nold)
            else:
                _detect_txns(cs, batch, now, nold)
            t += 0.4
            if i % 4 == 2:
                continue  # resolverCount <= 1 this batch: no adds
            off = 90 if i % 7 == 6 else 100
            ng = g.add_batch(cs, t + 1.0, offset_per_key=off)
            no = o.add_batch(batch, t + 1.0, offset_per_key=off)
            assert ng == no, (units, i, ng, no)
            assert g.queue_size() == len(o.queue)
            assert g.items() == o.items(), (units, i)
            if i % 3 == 0:
                g.poll(t)
                o.poll(t)
            if i == 8:
                g.attach(None)
                g.attach(cs)
        total = o.get_estimate(*ALL_KEYS)
        assert g.get_estimate(*ALL_KEYS) == total
        for front in (True, False):
            assert g.split_estimate(b"", b"\xff\xff", total // 3, front) == o.split_estimate(b"", b"\xff\xff",
                                                                                             total // 3, front)
        g.close()
    g = IopsSample(KEY_BYTES_PER_SAMPLE, seed=2)
    g.attach(cs)
    cs.close()  # (the engine goes first, as ~Resolver destroys the conflict set before its members)
    assert g.size() == 0
    g.close()


def test_add_metric_refuses_a_negative_total():
    """An entry's metric never goes below 0 (the prefix-sum index)."""
    s = IopsSample(1000)
    s.add_metric(b"a", 5)
    s.add_metric(b"a", -5)  # back to 0: erased
    with pytest.raises(Exception):
        s.add_metric(b"b", -1)
    with pytest.raises(Exception):
        s.add_metric(b"a", -1)
    s.close()
