"""CPU restatement of the Resolver's load-metrics sample -- TEST INFRASTRUCTURE ONLY.

Checker for foundationdb_amd/load_metrics.py (libfdbcs.so's fdbcs_sample_*):
only tests/ import it.

Follows
  * Resolver.actor.cpp:146-151   the addAndExpire loop (writes, then reads, of
                                 each transaction in batch order; metric =
                                 SAMPLE_OFFSET_PER_KEY + |begin|)
  * StorageMetrics.actor.h:98-182 TransientStorageMetricSample: roll (:103-105),
                                 addAndExpire (:108-113), poll (:150-164),
                                 add (:167-181)
  * StorageMetrics.actor.h:29-73 StorageMetricSample: getEstimate, splitEstimate
  * flow/IndexedSet.h:587-598 (addMetric), :1043-1063 (index), sumTo
  * fdbclient/FDBTypes.h:304-325 keyBetween; fdbclient/Knobs.cpp:57,60
    SPLIT_KEY_SIZE_LIMIT = KEY_SIZE_LIMIT / 2 = 5000

The roll: the reference draws g_random->random01() < metric / units from an
unseeded stream, so no recorded sample can be reproduced.  This build defines
draw `pos` of batch `seq` as mix64(seed + seq*C1 + pos*C2) mod units < metric
(load_metrics.hip), restated here with numpy's wrapping uint64 arithmetic.

Parity: the sample structure (getEstimate) is pinned by the reference's own
known-answer test, TEST_CASE("/fdbserver/StorageMetricSample/simple")
(StorageMetrics.actor.h:81-93), checked in tests/test_load_metrics.py.  The
roll and splitEstimate are unpinned by reference execution (the reference
is unbuildable here; its one splitEstimate assertion, :91, is
commented out).
"""
import bisect

import numpy as np

SPLIT_KEY_SIZE_LIMIT = 5000
_C1 = np.uint64(0xD1B54A32D192ED03)
_C2 = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def roll_hash(seed, seq, pos):
    """mix64 of the draw counter, vectorised over pos (uint64 array)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.uint64(seq) * _C1 + np.asarray(pos, dtype=np.uint64) * _C2
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def add_order_slots(batch):
    """Begin-key slots in the Resolver's addAndExpire order (Resolver.actor.cpp:
    146-151): for each transaction its writes, then its reads."""
    R = batch.R
    slots = []
    for t in range(batch.T):
        for w in range(int(batch.write_off[t]), int(batch.write_off[t + 1])):
            slots.append(2 * R + 2 * w)
        for r in range(int(batch.read_off[t]), int(batch.read_off[t + 1])):
            slots.append(2 * r)
    return np.asarray(slots, dtype=np.int64)


def roll_batch(batch, seed, seq, offset_per_key, units):
    """[(key bytes, amount)] for the sampled ranges of one batch, in add order."""
    slots = add_order_slots(batch)
    if slots.size == 0:
        return []
    lens = batch.key_len[slots].astype(np.int64)
    metric = offset_per_key + lens
    h = roll_hash(seed, seq, np.arange(slots.size, dtype=np.uint64))
    drawn = (h % np.uint64(units)).astype(np.int64) < metric
    amount = np.where(metric >= units, metric, np.where(drawn, units, 0))
    amount = np.where(metric <= 0, 0, amount)
    out = []
    kb = batch.key_bytes
    for i in np.nonzero(amount)[0]:
        s = int(slots[i])
        o = int(batch.key_off[s])
        out.append((kb[o:o + int(batch.key_len[s])].tobytes(), int(amount[i])))
    return out


def key_between(b, e):
    """keyBetween (fdbclient/FDBTypes.h:304-325)."""
    pos = 0
    mn = min(len(b), len(e))
    while pos < mn and pos < SPLIT_KEY_SIZE_LIMIT:
        if b[pos] != e[pos]:
            return e[:pos + 1]
        pos += 1
    if pos < SPLIT_KEY_SIZE_LIMIT and len(b) < len(e):
        return e[:pos + 1]
    return e


class SpecSample:
    """TransientStorageMetricSample over a sorted key list."""

    def __init__(self, units, seed=0):
        self.units = units
        self.seed = seed
        self.seq = 0
        self.keys = []      # sorted
        self.metric = {}    # key -> metric
        self.queue = []     # (expiration, key, delta), FIFO

    # IndexedSet::addMetric + erase at zero
    def add_metric(self, k, m):
        v = self.metric.get(k, 0) + m
        if v == 0:
            if k in self.metric:
                del self.metric[k]
                self.keys.pop(bisect.bisect_left(self.keys, k))
        elif k in self.metric:
            self.metric[k] = v
        else:
            self.metric[k] = v
            bisect.insort(self.keys, k)

    def add_batch(self, batch, expiration, offset_per_key=100):
        seq = self.seq
        self.seq += 1
        rolled = roll_batch(batch, self.seed, seq, offset_per_key, self.units) if batch.T else []
        for k, x in rolled:
            self.add_metric(k, x)
            self.queue.append((expiration, k, -x))
        return len(rolled)

    def poll(self, now):
        while self.queue and self.queue[0][0] <= now:
            _, k, d = self.queue.pop(0)
            assert d != 0
            self.add_metric(k, d)

    def _prefix(self):
        p = [0]
        for k in self.keys:
            p.append(p[-1] + self.metric[k])
        return p

    def sum_to(self, i, p=None):
        return (p or self._prefix())[i]

    def get_estimate(self, b, e):
        p = self._prefix()
        return p[bisect.bisect_left(self.keys, e)] - p[bisect.bisect_left(self.keys, b)]

    def index(self, m, p):
        # first x with m < sumTo(x + 1), or end
        for i in range(len(self.keys)):
            if m < p[i + 1]:
                return i
        return len(self.keys)

    def split_estimate(self, rb, re, offset, front=True):
        """StorageMetricSample::splitEstimate (StorageMetrics.actor.h:38-73)."""
        p = self._prefix()
        K = self.keys
        n = len(K)
        if front:
            anchor = p[bisect.bisect_left(K, rb)] + offset
        else:
            anchor = p[bisect.bisect_left(K, re)] - offset
        fwd = self.index(anchor, p)
        if fwd == n or K[fwd] >= re:
            return re
        if not front and K[fwd] <= rb:
            return rb
        bck = fwd
        while (fwd != n and K[fwd] < re) or (bck != 0 and K[bck] > rb):
            if bck != 0 and K[bck] > rb:
                it = bck
                bck -= 1
                split = key_between(max(K[bck], rb) if bck != 0 else rb, K[it])
                if not front or (self.get_estimate(rb, split) > 0 and len(split) <= SPLIT_KEY_SIZE_LIMIT):
                    return split
            if fwd != n and K[fwd] < re:
                it = fwd + 1
                split = key_between(K[fwd], min(K[it], re) if it != n else re)
                if front or (self.get_estimate(split, re) > 0 and len(split) <= SPLIT_KEY_SIZE_LIMIT):
                    return split
                fwd = it
        return re if front else rb

    def items(self):
        return [(k, self.metric[k]) for k in self.keys]
