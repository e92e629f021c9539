"""CPU model of one shard of the exact sharded mode (test infrastructure).

Implements the interface of ``foundationdb_amd.sharded.Shard`` (check / apply
/ compact / clear / history) over a Python sorted list, so the host protocol
(``plan_compaction``, ``carry_ins``, the removalKey broadcast, the gloo/RCCL
exchanges of ``DistShardedConflictSet``) runs without a GPU and is checked
against the single-resolver oracle (``oracle.spec``).  Each step restates
SURVEY.md §8e protocol A for the keys ``[lo, hi)``:

- check: a read clipped to the shard; valueBefore of a clipped begin that has
  no earlier boundary in the shard is the carry-in (SkipList.cpp:755-837 over
  the shard's part of the key space).
- apply: the ordered decision and the combine over the whole batch
  (SkipList.cpp:1133-1153, :1320-1337), then the merge clipped: a begin node
  only where b lies in the shard, an end node only where e does
  (SkipList.cpp:511-522).
- compact: removeBefore's rule (SkipList.cpp:665-702) over the shard's part of
  the global window.
"""
import ctypes as C
from bisect import bisect_left

import numpy as np

from foundationdb_amd.batch import PackedBatch

INT64_MIN = -(1 << 63)


def _bytes_at(ptr, n):
    return np.ctypeslib.as_array((C.c_uint8 * max(1, n)).from_address(ptr))[:n]


class ModelShard:
    def __init__(self, lo, hi, device=-1, v0=0, max_history=0, sparse=False):
        self.lo, self.hi = lo, hi
        self.sparse = sparse
        self.edges = []   # protocol B: this shard's (reader, earlier writer) pairs
        self.gedges = []  # the union over the shards
        self.v0 = v0  # carry-in
        self.keys, self.vers = [], []
        self.oldest = 0
        self.rk = b""

    def _in(self, k):
        return (self.lo is None or k >= self.lo) and (self.hi is None or k < self.hi)

    def _txns(self, view):
        b = PackedBatch.from_view(view)
        return b.txns()

    def _value_before(self, k):
        i = bisect_left(self.keys, k)
        return self.vers[i - 1] if i > 0 else self.v0

    def check(self, view, now, new_oldest, carry, dev_hist):
        self.v0 = carry
        txns = self._txns(view)
        out = _bytes_at(dev_hist, len(txns))
        self.edges = []
        if self.sparse:  # overlaps of this shard's ranges (present whole: ranges arrive unclipped)
            for t, (snap, reads, _w) in enumerate(txns):
                for u in range(t):
                    if any(rb < we and wb < re_ for rb, re_ in reads for wb, we in txns[u][2]):
                        self.edges.append((t, u))
        for t, (snap, reads, _w) in enumerate(txns):
            out[t] = 0
            if snap < self.oldest and reads:
                out[t] = 2
                continue  # tooOld: not checked (SkipList.cpp:985)
            for b, e in reads:
                if self.lo is not None and b < self.lo:
                    b = self.lo
                if self.hi is not None and e > self.hi:
                    e = self.hi
                if b >= e:
                    continue
                i = bisect_left(self.keys, b)
                m = self.vers[i] if i < len(self.keys) and self.keys[i] == b else self._value_before(b)
                j = bisect_left(self.keys, e)
                for x in range(i, j):
                    m = max(m, self.vers[x])
                if m > snap:
                    out[t] = 1

    def apply(self, view, now, new_oldest, carry, removal_key, dev_hist, dev_verdict):
        self.v0 = carry
        if removal_key is not None:
            self.rk = removal_key
        txns = self._txns(view)
        T = len(txns)
        flags = _bytes_at(dev_hist, T).copy()
        too_old = [flags[t] == 2 for t in range(T)]
        conflict = [flags[t] != 0 for t in range(T)]
        if self.sparse:  # the ordered decision over the global edges
            src = {}
            for t, u in self.gedges:
                src.setdefault(t, []).append(u)
            for t in range(T):
                if not conflict[t]:
                    conflict[t] = any(not conflict[u] for u in src.get(t, ()))
        else:
            acc = []
            for t, (_s, reads, writes) in enumerate(txns):
                if conflict[t]:
                    continue
                c = any(rb < we and wb < re_ for rb, re_ in reads for wb, we in acc)
                conflict[t] = c
                if not c:
                    acc.extend(writes)
        verdict = _bytes_at(dev_verdict, T)
        for t in range(T):
            verdict[t] = 2 if not conflict[t] else (1 if too_old[t] else 0)
        pts = []
        for t, (_s, _r, writes) in enumerate(txns):
            if not conflict[t]:
                for b, e in writes:
                    pts += [(b, 1), (e, 0)]
        pts.sort()
        combined, active = [], 0
        for k, is_begin in pts:
            if is_begin:
                active += 1
                if active == 1:
                    combined.append([k, None])
            else:
                active -= 1
                if active == 0:
                    combined[-1][1] = k
        for b, e in reversed(combined):
            if (self.hi is not None and b >= self.hi) or (self.lo is not None and e < self.lo):
                continue
            if self._in(e):
                j = bisect_left(self.keys, e)
                if not (j < len(self.keys) and self.keys[j] == e):
                    vb = self._value_before(e)
                    self.keys.insert(j, e)
                    self.vers.insert(j, vb)
            i = bisect_left(self.keys, b)
            j = bisect_left(self.keys, e)
            del self.keys[i:j]
            del self.vers[i:j]
            if self._in(b):
                self.keys.insert(i, b)
                self.vers.insert(i, now)
        H = len(self.keys)
        g0 = bisect_left(self.keys, self.rk) if new_oldest > self.oldest else -1
        own = sum(1 for b, _e in combined if self._in(b))
        return H, g0, (self.vers[-1] if H else INT64_MIN), own

    def edge_count(self):
        return len(self.edges)

    def get_edges(self, et_ptr, eu_ptr, n):
        et = np.ctypeslib.as_array((C.c_int32 * max(1, n)).from_address(et_ptr))
        eu = np.ctypeslib.as_array((C.c_int32 * max(1, n)).from_address(eu_ptr))
        for i, (t, u) in enumerate(self.edges[:n]):
            et[i], eu[i] = t, u

    def set_edges(self, et_ptr, eu_ptr, n):
        et = np.ctypeslib.as_array((C.c_int32 * max(1, n)).from_address(et_ptr))[:n]
        eu = np.ctypeslib.as_array((C.c_int32 * max(1, n)).from_address(eu_ptr))[:n]
        self.gedges = list(zip(et.tolist(), eu.tolist()))

    def compact(self, part, new_oldest, key_index=-1):
        a, b, keep_first, prev = part
        key = self.keys[key_index] if key_index >= 0 else None
        keep_k, keep_v = self.keys[:a], self.vers[:a]
        for i in range(a, b):
            pv = self.vers[i - 1] if i > 0 else prev
            if (i == a and keep_first) or self.vers[i] >= new_oldest or pv >= new_oldest:
                keep_k.append(self.keys[i])
                keep_v.append(self.vers[i])
        self.keys = keep_k + self.keys[b:]
        self.vers = keep_v + self.vers[b:]
        self.oldest = max(self.oldest, new_oldest)
        return len(self.keys), (self.vers[-1] if self.keys else INT64_MIN), key

    def clear(self, v):
        self.keys, self.vers = [], []
        self.v0 = v

    def history(self):
        return list(zip(self.keys, self.vers))

    def close(self):
        pass
