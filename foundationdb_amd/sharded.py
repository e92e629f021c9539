"""Exact sharded conflict set: one Resolver over G GPUs (SURVEY.md §8e protocol A).

The north star's node layout.

- GPU g holds the history of the keys in ``[bounds[g-1], bounds[g])``.
- Every GPU receives the whole batch.
- The host exchanges three times per batch.

The result equals one ``ConflictSet`` (a single Resolver,
Resolver.actor.cpp:140-153) bit for bit:

- verdicts;
- the concatenated history;
- removalKey and oldestVersion.

Per batch (the step numbers are SURVEY.md §8e's), two exchanges:

1-2. ``fdbcs_shard_check``: each shard checks every read clipped to its keys.
     valueBefore of a clipped begin is the shard's carry-in: the version of
     the nearest earlier non-empty shard's last boundary after the previous
     batch's MERGE (or the header version v0).  The previous compaction can
     change that value only between two versions below oldestVersion, and a
     checked read's snapshot is >= oldestVersion, so the check cannot tell.
3.   Exchange 1, one MAX all-reduce of a byte buffer: the per-transaction
     history-conflict flags (T bytes) followed by one slot per shard that
     only its owner fills (a MAX over zeros is an all-gather): the shard's
     (H, last version) after the previous compaction, and the new removalKey
     from the shard that read it.
4-5. ``fdbcs_shard_apply`` with the exact carry-in from those slots: an
     identical decision and combine on every shard, then the shard's part of
     the merge (a begin node only where the real begin lies, an end node only
     in the shard holding the end; an end node with no boundary below it in
     the shard takes the exact carry-in).
6.   Exchange 2, an all-gather of (H, first index >= removalKey, last
     version) after the merge.  Compaction over global boundary indices: the
     window starts at the first boundary >= removalKey anywhere and spans
     ``3 * |combined| + 10`` boundaries; each shard removes in its part, and
     the "previous node" crosses shard edges.  The shard holding the window's
     end reads the new removalKey (delivered in the next exchange 1).
7.   Carry-ins for the next check from exchange 2's last versions.

Two exchange back ends share the logic below:

- ``ShardedConflictSet`` runs all shards in one process (on one or several
  devices). Tests use it.
- ``DistShardedConflictSet`` is one shard per rank over torch.distributed:
  RCCL over xGMI, or gloo on CPU.

``_Proto`` holds one shard's protocol state; both back ends drive it.
"""
import ctypes as C
import time

import numpy as np

from . import _abi
from ._abi import check
from .conflict_set import ConflictSet

INT64_MIN = -(1 << 63)


def plan_compaction(infos, n_comb):
    """The global compaction window, cut per shard.

    infos[g] = (H_g, g0_g, last_version_g) after the merge.  g0_g is the
    index of the shard's first boundary >= removalKey (H_g if none).

    Returns ``(parts, owner)``:

    - ``parts[g] = (a, b, keep_first, prev_version)``, local indices.
    - ``owner = (g, local_index)`` of the boundary that becomes removalKey,
      or None for "" (the scan reached the end).

    Restates SkipList.cpp:665-702 over the concatenated shards.
    """
    G = len(infos)
    offs, tot = [], 0
    for H, _g0, _last in infos:
        offs.append(tot)
        tot += H
    G0 = tot
    for g, (H, g0, _last) in enumerate(infos):
        if g0 < H:
            G0 = offs[g] + g0
            break
    parts = [(0, 0, 0, 0)] * G
    if G0 >= tot:
        return parts, None
    G1 = min(tot, G0 + 3 * n_comb + 10)
    prev_last = None  # last version of the nearest earlier non-empty shard
    for g, (H, _g0, last) in enumerate(infos):
        a = min(max(G0 - offs[g], 0), H)
        b = min(max(G1 - offs[g], 0), H)
        keep_first = 1 if offs[g] <= G0 < offs[g] + H else 0
        prev = prev_last if (a == 0 and a < b and not keep_first) else 0
        parts[g] = (a, b, keep_first, prev if prev is not None else 0)
        if H:
            prev_last = last
    owner = None
    if G1 < tot:
        for g, (H, _g0, _last) in enumerate(infos):
            if offs[g] <= G1 < offs[g] + H:
                owner = (g, G1 - offs[g])
                break
    return parts, owner


KEY_INLINE = 32  # removalKeys up to this length travel inside exchange 1
SLOT_WORDS = 4 + KEY_INLINE // 8  # H, last version, key length (-1: none), edges (protocol B), key words
EDGE_INLINE = 1024  # protocol B: overlap edges per shard carried inside exchange 1 (more: a separate all-gather)


def _pack_key(key):
    raw = key.ljust(KEY_INLINE, b"\0")
    return [int.from_bytes(raw[i:i + 8], "little", signed=True) for i in range(0, KEY_INLINE, 8)]


def _unpack_key(words, n):
    return b"".join(int(w).to_bytes(8, "little", signed=True) for w in words)[:n]


def carry_ins(v0, hl):
    """Carry-in of every shard from (H_g, last_version_g): step 7."""
    out, cur = [], v0
    for H, last in hl:
        out.append(cur)
        if H:
            cur = last
    return out




class Shard:
    """One engine holding the keys [lo, hi) (None: unbounded)."""

    def __init__(self, lo, hi, device=-1, v0=0, max_history=0, sparse=False, tail_arena_bytes=0):
        self.cs = ConflictSet(v0=v0, device=device, max_history=max_history, tail_arena_bytes=tail_arena_bytes)
        self._lib = self.cs._lib
        lo_b, hi_b = lo or b"", hi or b""
        check(self._lib.fdbcs_set_shard(self.cs.handle, lo_b, len(lo_b), int(lo is not None), hi_b, len(hi_b),
                                        int(hi is not None)), "set_shard")
        if sparse:
            check(self._lib.fdbcs_shard_set_protocol(self.cs.handle, 1), "shard_set_protocol")
        self.lo, self.hi = lo, hi
        self._key = (C.c_uint8 * _abi.MAX_KEY)()

    def check(self, dev_view, now, new_oldest, carry, dev_hist):
        check(self._lib.fdbcs_shard_check(self.cs.handle, C.byref(dev_view), now, new_oldest, carry, dev_hist),
              "shard_check")

    def apply(self, dev_view, now, new_oldest, carry, removal_key, dev_hist, dev_verdict):
        info = (C.c_int64 * 4)()
        rk = removal_key if removal_key is not None else b""
        n = len(rk) if removal_key is not None else -1
        check(self._lib.fdbcs_shard_apply(self.cs.handle, C.byref(dev_view), now, new_oldest, carry, rk, n, dev_hist,
                                          dev_verdict, info), "shard_apply")
        return tuple(info)

    def edge_count(self):
        n = self._lib.fdbcs_shard_edge_count(self.cs.handle)
        if n < 0:
            check(int(n), "shard_edge_count")
        return int(n)

    def get_edges(self, et_ptr, eu_ptr, n):
        check(self._lib.fdbcs_shard_get_edges(self.cs.handle, et_ptr, eu_ptr, n), "shard_get_edges")

    def set_edges(self, et_ptr, eu_ptr, n):
        check(self._lib.fdbcs_shard_set_edges(self.cs.handle, et_ptr, eu_ptr, n), "shard_set_edges")

    def compact(self, part, new_oldest, key_index=-1):
        a, b, keep_first, prev = part
        info = (C.c_int64 * 3)()
        check(self._lib.fdbcs_shard_compact(self.cs.handle, a, b, keep_first, prev, new_oldest, key_index, self._key,
                                            _abi.MAX_KEY, info), "shard_compact")
        key = bytes(self._key[:info[2]]) if info[2] >= 0 else None
        return info[0], info[1], key

    def clear(self, v):
        self.cs.clear(v)

    def history(self):
        return self.cs.history()

    def close(self):
        self.cs.close()


def _shard_ranges(bounds):
    edges = [None] + list(bounds) + [None]
    return [(edges[g], edges[g + 1]) for g in range(len(bounds) + 1)]


def _device(torch, d):
    return torch.device("cpu") if d is None or d < 0 else torch.device("cuda", d)


def _sync(torch, dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class _Proto:
    """Protocol state of shard g (module docstring, steps 1-7)."""

    def __init__(self, shard, g, v0):
        self.shard, self.g = shard, g
        self.v0 = v0                  # header version: the carry-in of a shard with nothing below it
        self.carry_check = v0         # carry-in after the previous merge (step 7)
        self.slot = (0, INT64_MIN, -1, b"")  # after the previous compaction: H, last, removalKey read here
        self.rk_owner = None          # shard whose slot holds the pending removalKey (-1: ""; None: unchanged)
        self.rk = b""                 # removalKey as delivered
        self.oldest = 0

    def slot_words(self, edges=0):
        H, last, n, key = self.slot
        return [H, last, n, edges] + _pack_key(key if 0 <= n <= KEY_INLINE else b"")

    def check(self, view, now, new_oldest, hist_ptr):
        self.shard.check(view, now, new_oldest, self.carry_check, hist_ptr)

    def pending_key(self, slots, long_key=None):
        """The removalKey the previous compaction produced, from exchange 1's slots (None: unchanged)."""
        if self.rk_owner is None:
            return None
        if self.rk_owner < 0:
            return b""
        n = slots[self.rk_owner][2]
        return _unpack_key(slots[self.rk_owner][4:], n) if n <= KEY_INLINE else long_key

    def apply(self, view, now, new_oldest, slots, hist_ptr, verdict_ptr, long_key=None):
        carry = carry_ins(self.v0, [(w[0], w[1]) for w in slots])[self.g]
        rk = self.pending_key(slots, long_key)
        if rk is not None:
            self.rk, self.rk_owner = rk, None
        H, g0, last, n_own = self.shard.apply(view, now, new_oldest, carry, rk, hist_ptr, verdict_ptr)
        return (H, g0, last), n_own

    def compact(self, infos, n_comb, new_oldest):
        if new_oldest > self.oldest:  # step 6
            parts, owner = plan_compaction(infos, n_comb)
            ki = owner[1] if owner is not None and owner[0] == self.g else -1
            Hn, lastn, key = self.shard.compact(parts[self.g], new_oldest, ki)
            self.slot = (Hn, lastn, len(key) if key is not None else -1, key or b"")
            self.rk_owner = owner[0] if owner is not None else -1
            self.oldest = new_oldest
        else:
            H, _g0, last = infos[self.g]
            self.slot = (H, last, -1, b"")
        self.carry_check = carry_ins(self.v0, [(x[0], x[2]) for x in infos])[self.g]  # step 7

    def clear(self, v):
        """clearConflictSet (SkipList.cpp:957-959): empty history, header version v; oldestVersion and
        removalKey (even one still in flight) are kept."""
        self.shard.clear(v)
        self.v0 = self.carry_check = v
        self.slot = (0, INT64_MIN) + self.slot[2:]


class ShardedConflictSet:
    """All G shards in this process (on one or several devices): the exchanges
    are a device reduction and host lists.  ``shard_factory`` builds a shard
    (tests pass a CPU model of the same interface)."""

    def __init__(self, bounds, devices=None, v0=0, max_history=0, shard_factory=Shard, sparse=False, **shard_kw):
        import torch

        self.torch = torch
        self.bounds = list(bounds)
        self.sparse = sparse  # protocol B: shard-local ranges, exchanged overlap edges
        ranges = _shard_ranges(bounds)
        if devices is None:
            d = torch.cuda.current_device() if torch.cuda.is_available() else -1
            devices = [d] * len(ranges)
        assert len(devices) == len(ranges)
        self.devices = [_device(torch, d) for d in devices]
        self.protos = [_Proto(shard_factory(lo, hi, device=d, v0=v0, max_history=max_history, sparse=sparse,
                                            **shard_kw), g, v0)
                       for g, ((lo, hi), d) in enumerate(zip(ranges, devices))]
        self.shards = [p.shard for p in self.protos]

    def clear(self, v):
        for p in self.protos:
            p.clear(v)

    def detect_device(self, views, now, new_oldest, verdict):
        """views[g]: the batch in shard g's device memory; verdict: uint8 tensor [>= T] on devices[0]."""
        torch = self.torch
        T = views[0].txn_count
        hs = [torch.empty(max(1, T), dtype=torch.uint8, device=d) for d in self.devices]
        for d in set(self.devices):
            _sync(torch, d)
        for p, v, h in zip(self.protos, views, hs):  # steps 1-2
            p.check(v, now, new_oldest, h.data_ptr())
        flags = torch.stack([h.to(self.devices[0]) for h in hs]).amax(0)  # step 3: MAX over shards
        slots = [p.slot_words() for p in self.protos]
        et = eu = None
        if self.sparse:  # protocol B: the union of the shards' overlap edges
            parts = []
            for p, d in zip(self.protos, self.devices):
                n = p.shard.edge_count()
                a = torch.empty(max(1, n), dtype=torch.int32, device=d)
                b = torch.empty(max(1, n), dtype=torch.int32, device=d)
                p.shard.get_edges(a.data_ptr(), b.data_ptr(), n)
                parts.append((a[:n].to(self.devices[0]), b[:n].to(self.devices[0])))
            et = torch.cat([a for a, _ in parts] + [torch.zeros(1, dtype=torch.int32, device=self.devices[0])])
            eu = torch.cat([b for _, b in parts] + [torch.zeros(1, dtype=torch.int32, device=self.devices[0])])
        n_edges = et.numel() - 1 if et is not None else 0
        infos, n_comb = [], 0
        for g, (p, v) in enumerate(zip(self.protos, views)):  # steps 4-5
            f = flags.to(self.devices[g])
            out = verdict if g == 0 else torch.empty(max(1, T), dtype=torch.uint8, device=self.devices[g])
            if et is not None:
                ge, gu = et.to(self.devices[g]), eu.to(self.devices[g])
                _sync(torch, self.devices[g])
                p.shard.set_edges(ge.data_ptr(), gu.data_ptr(), n_edges)
            _sync(torch, self.devices[g])
            o = p.rk_owner
            long_key = self.protos[o].slot[3] if o is not None and o >= 0 else None
            info, n_own = p.apply(v, now, new_oldest, slots, f.data_ptr(), out.data_ptr(), long_key)
            infos.append(info)
            n_comb += n_own  # |combined ranges| of the whole batch: each begins in exactly one shard
        for p in self.protos:  # steps 6-7
            p.compact(infos, n_comb, new_oldest)

    def detect_packed(self, batch, now, new_oldest):
        """A host PackedBatch through the sharded path; returns the verdict bytes (numpy)."""
        from .batch import DeviceBatch

        verdict = self.torch.empty(max(1, batch.T), dtype=self.torch.uint8, device=self.devices[0])
        if self.sparse:  # each shard gets the ranges intersecting its keys (all transactions)
            from .resolvers import KeyRangeResolvers

            kr = KeyRangeResolvers(self.bounds)
            subs = [kr.split(batch, g, keep_all=True)[0] for g in range(len(self.devices))]
            staged = [DeviceBatch(sb, d) for sb, d in zip(subs, self.devices)]
            self.detect_device([x.view for x in staged], now, new_oldest, verdict)
            return verdict[:batch.T].cpu().numpy()
        staged = {}
        for d in self.devices:
            if d not in staged:
                staged[d] = DeviceBatch(batch, d)
        self.detect_device([staged[d].view for d in self.devices], now, new_oldest, verdict)
        return verdict[:batch.T].cpu().numpy()

    @property
    def oldest_version(self):
        return self.protos[0].oldest

    def history(self):
        out = []
        for s in self.shards:
            out += s.history()
        return out

    def removal_key(self):
        p = self.protos[0]
        rk = p.pending_key([q.slot_words() for q in self.protos], self._owner_key(p.rk_owner))
        return p.rk if rk is None else rk

    def _owner_key(self, o):
        return self.protos[o].slot[3] if o is not None and o >= 0 else None

    def close(self):
        for s in self.shards:
            s.close()


class DistShardedConflictSet:
    """One shard per torch.distributed rank (RCCL over xGMI on MI355X, gloo on CPU).

    Per batch: the engine's check, one MAX all-reduce (flags + slots), the
    engine's apply, one all-gather of three integers, the engine's compaction.
    """

    def __init__(self, bounds, rank, world, device, v0=0, max_history=0, group=None, shard_factory=Shard,
                 sparse=False, edge_inline=EDGE_INLINE):
        import torch
        import torch.distributed as dist

        assert len(bounds) + 1 == world
        self.torch, self.dist, self.group = torch, dist, group
        self.rank, self.world = rank, world
        self.bounds = list(bounds)
        self.sparse = sparse  # protocol B: this rank receives only its ranges; overlap edges are all-gathered
        self.ei = max(1, edge_inline)
        self.device = _device(torch, device)
        lo, hi = _shard_ranges(bounds)[rank]
        self.shard = shard_factory(lo, hi, device=device, v0=v0, max_history=max_history, sparse=sparse)
        self.proto = _Proto(self.shard, rank, v0)
        backend = dist.get_backend(group)
        self.coll_dev = self.device if backend == "nccl" else torch.device("cpu")
        self._T = -1
        self.phase_s = None

    def clear(self, v):
        self.proto.clear(v)

    def _buffers(self, T):
        if T != self._T:
            torch = self.torch
            nT8 = (max(1, T) + 7) // 8 * 8
            n = nT8 + self.world * SLOT_WORDS * 8 + (self.world * 2 * self.ei * 4 if self.sparse else 0)
            self._h = torch.empty(max(1, T), dtype=torch.uint8, device=self.device)
            self._x1 = torch.zeros(n, dtype=torch.uint8, device=self.coll_dev)
            self._eoff = nT8 + self.world * SLOT_WORDS * 8
            self._eb = torch.zeros(2 * self.ei, dtype=torch.int32, device=self.device)
            self._T = T
        return self._h, self._x1

    def detect_device(self, view, now, new_oldest, verdict):
        """view: the whole batch in this rank's device memory; verdict: uint8 tensor [>= T] there."""
        torch, dist, p = self.torch, self.dist, self.proto
        tick = self._tick
        tick(None)
        T = view.txn_count
        h, x1 = self._buffers(T)
        nT = max(1, T)
        _sync(torch, self.device)
        p.check(view, now, new_oldest, h.data_ptr())  # steps 1-2 (synchronous)
        tick("check")
        # exchange 1: flags + this shard's slot, zeros elsewhere; MAX all-reduce
        n_edges = self.shard.edge_count() if self.sparse else 0
        mine = np.zeros(self.world * SLOT_WORDS, np.int64)
        mine[self.rank * SLOT_WORDS:(self.rank + 1) * SLOT_WORDS] = p.slot_words(n_edges)
        so, eo = self._eoff - self.world * SLOT_WORDS * 8, self._eoff
        x1[so:eo].copy_(torch.from_numpy(mine.view(np.uint8)))
        x1[:nT].copy_(h)
        if self.sparse:  # protocol B: up to self.ei edges per shard ride in this all-reduce too
            x1[eo:].zero_()
            if 0 < n_edges <= self.ei:
                self.shard.get_edges(self._eb.data_ptr(), self._eb[self.ei:].data_ptr(), n_edges)
                w = 2 * self.ei * 4
                x1[eo + self.rank * w:eo + (self.rank + 1) * w].copy_(self._eb.view(torch.uint8))
        dist.all_reduce(x1, op=dist.ReduceOp.MAX, group=self.group)
        slots = torch.empty(self.world * SLOT_WORDS * 8, dtype=torch.uint8)
        slots.copy_(x1[so:eo])
        slots = slots.numpy().view(np.int64).reshape(self.world, SLOT_WORDS).tolist()
        if x1.device != self.device:
            h.copy_(x1[:nT])
            fl = h
        else:
            fl = x1
        if self.sparse:  # protocol B: the union of the overlap edges (counts came in the slots)
            counts = [int(w[3]) for w in slots]
            if sum(counts) == 0:
                pass  # (no overlaps anywhere: this shard's own empty list is the global one)
            elif max(counts) <= self.ei:
                ed = x1[eo:].view(torch.int32).view(self.world, 2, self.ei).to(self.device)
                et = torch.cat([ed[g, 0, :counts[g]] for g in range(self.world)] + [ed.new_zeros(1)])
                eu = torch.cat([ed[g, 1, :counts[g]] for g in range(self.world)] + [ed.new_zeros(1)])
                _sync(torch, self.device)
                self.shard.set_edges(et.data_ptr(), eu.data_ptr(), sum(counts))
                self._edges_keep = (et, eu)
            else:  # a long list somewhere: one more all-gather
                self._exchange_edges(counts, n_edges)
        _sync(torch, self.device)  # the engine reads the flags on its own stream
        tick("exchange1")
        long_key = None
        o = p.rk_owner
        if o is not None and o >= 0 and slots[o][2] > KEY_INLINE:
            long_key = self._broadcast_key(o, p.slot[3] if o == self.rank else b"")
        info, n_own = p.apply(view, now, new_oldest, slots, fl.data_ptr(), verdict.data_ptr(), long_key)  # 4-5
        tick("apply")
        got = self._allgather(list(info) + [n_own])  # exchange 2
        infos = [tuple(x[:3]) for x in got]
        n_comb = sum(x[3] for x in got)  # each combined range begins in exactly one shard
        tick("exchange2")
        p.compact(infos, n_comb, new_oldest)  # steps 6-7
        tick("compact")

    def _exchange_edges(self, counts, n_mine):
        """One all-gather of every shard's (reader, earlier writer) pairs, padded
        to the longest list; their concatenation replaces this shard's own."""
        torch, dist = self.torch, self.dist
        m = max(1, max(counts))
        buf = torch.zeros(2 * m, dtype=torch.int32, device=self.device)
        self.shard.get_edges(buf.data_ptr(), buf[m:].data_ptr(), n_mine)
        send = buf.to(self.coll_dev)
        outs = [torch.empty_like(send) for _ in range(self.world)]
        dist.all_gather(outs, send, group=self.group)
        out = torch.stack(outs).view(self.world, 2, m).to(self.device)
        et = torch.cat([out[g, 0, :counts[g]] for g in range(self.world)] + [out.new_zeros(1)])
        eu = torch.cat([out[g, 1, :counts[g]] for g in range(self.world)] + [out.new_zeros(1)])
        _sync(torch, self.device)
        self.shard.set_edges(et.data_ptr(), eu.data_ptr(), sum(counts))
        self._edges_keep = (et, eu)  # (alive until the engine's copy has run)

    def split(self, batch):
        """This rank's input under protocol B: every transaction, only the ranges
        intersecting its keys (the proxy's per-resolver split keeping batch
        indices); the whole batch under protocol A."""
        if not self.sparse:
            return batch
        from .resolvers import KeyRangeResolvers

        return KeyRangeResolvers(self.bounds).split(batch, self.rank, keep_all=True)[0]

    def detect_packed(self, batch, now, new_oldest):
        from .batch import DeviceBatch

        db = DeviceBatch(self.split(batch), self.device)
        verdict = self.torch.empty(max(1, batch.T), dtype=self.torch.uint8, device=self.device)
        self.detect_device(db.view, now, new_oldest, verdict)
        return verdict[:batch.T].cpu().numpy()

    def enable_phase_timing(self, on=True):
        """Accumulate host wall time per protocol phase (``phase_s``)."""
        self.phase_s = {} if on else None

    def _tick(self, name):
        if self.phase_s is None:
            return
        t = time.perf_counter()
        if name is not None:
            self.phase_s[name] = self.phase_s.get(name, 0.0) + t - self._t
        self._t = t

    def _broadcast_key(self, owner, key):
        """A removalKey too long for exchange 1's slot, from the shard that read it."""
        torch, dist = self.torch, self.dist
        buf = torch.zeros(_abi.MAX_KEY + 4, dtype=torch.uint8)
        if owner == self.rank:
            buf[:4 + len(key)] = torch.frombuffer(bytearray(len(key).to_bytes(4, "little") + key), dtype=torch.uint8)
        buf = buf.to(self.coll_dev)
        dist.broadcast(buf, src=owner, group=self.group)
        raw = buf.cpu().numpy()
        n = int.from_bytes(raw[:4].tobytes(), "little")
        return raw[4:4 + n].tobytes()

    def _allgather(self, vals):
        torch, dist = self.torch, self.dist
        t = torch.tensor(vals, dtype=torch.int64, device=self.coll_dev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return torch.stack(out).cpu().tolist()  # (one device-to-host copy, not one per rank)

    @property
    def oldest_version(self):
        return self.proto.oldest

    def history(self):
        return self.shard.history()

    def history_size(self):
        return self.shard.cs.history_size()

    def removal_key(self):
        """The global removalKey (collective when the last compaction's key is still in flight)."""
        p = self.proto
        if p.rk_owner is None:
            return p.rk
        if p.rk_owner < 0:
            return b""
        return self._broadcast_key(p.rk_owner, p.slot[3] if p.rk_owner == self.rank else b"")

    def close(self):
        self.shard.close()


class _LocalEngine(ConflictSet):
    """A non-owning view of the engine inside an fdbcs_sharded (its shard's history)."""

    def __init__(self, lib, handle):
        self._lib = lib
        self._h = C.c_void_p(handle)

    def close(self):
        self._h = None  # (owned by the sharded set)


class ShardedResolver:
    """``fdbcs_sharded`` (include/fdbcs.h): one exact Resolver over G GPUs
    behind the C ABI, one instance per rank (SURVEY.md §8e protocol A).

    The per-batch protocol of this module's docstring runs inside libfdbcs on
    the engine's stream; carry-ins, the compaction plan and removalKey's owner
    are computed on the device, and the host waits once per batch, for the
    verdicts.  Exchanges: RCCL (``comm_id`` from ``unique_id()`` on rank 0,
    shared by the caller; one GPU per rank), or host collectives over a
    torch.distributed ``group`` (gloo) -- the multi-process tests on one GPU.
    """

    PROTOCOLS = {"a": 0, "b": 1}  # FDBCS_PROTOCOL_A / _B
    sharded = True  # (workload.ResolverRun: the fdbcs_sharded loop)
    PRESPLIT = 1                  # FDBCS_SHARD_PRESPLIT

    def __init__(self, bounds, rank, world, device=0, v0=0, max_history=0, comm_id=None, group=None, protocol="a",
                 presplit=False, tail_arena_bytes=0):
        """protocol "b": this rank takes only the ranges intersecting its keys
        (fdbcs_sharded_batch_add filters them unless ``presplit``; the packed
        and device paths take the rank's fdbcs_split_batch_keep_all share)."""
        assert len(bounds) + 1 == world
        self._lib = _abi.lib()
        self.rank, self.world = rank, world
        self.bounds = list(bounds)
        self.protocol = protocol
        kb = b"".join(bounds)
        offs = np.cumsum([0] + [len(b) for b in bounds])[:-1].astype(np.uint64) if bounds else np.zeros(1, np.uint64)
        lens = np.array([len(b) for b in bounds] or [0], np.uint32)
        kb_arr = np.frombuffer(kb + b"\0", np.uint8).copy()
        cfg = _abi.Config(device=device, max_history=max_history, tail_arena_bytes=tail_arena_bytes)
        h = C.c_void_p()
        ops_p = None
        cid = None
        if comm_id is None:
            self._ops = self._host_ops(group)
            ops_p = C.byref(self._ops)
        else:
            cid = (C.c_uint8 * _abi.COMM_ID_BYTES).from_buffer_copy(bytes(comm_id))
        check(self._lib.fdbcs_sharded_create(C.byref(h), rank, world, kb_arr.ctypes.data, offs.ctypes.data,
                                             lens.ctypes.data, v0, C.byref(cfg), cid, ops_p), "fdbcs_sharded_create")
        self._h = h
        self.local = _LocalEngine(self._lib, self._lib.fdbcs_sharded_local(h))
        check(self._lib.fdbcs_sharded_set_protocol(h, self.PROTOCOLS[protocol], self.PRESPLIT if presplit else 0),
              "fdbcs_sharded_set_protocol")

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * _abi.COMM_ID_BYTES)()
        check(_abi.lib().fdbcs_comm_unique_id(buf), "fdbcs_comm_unique_id")
        return bytes(buf)

    def _host_ops(self, group):
        import torch
        import torch.distributed as dist

        world = self.world

        def allreduce(_ctx, buf, n):
            try:
                t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(n,)))  # (in place)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
                return 0
            except Exception:  # (an exception must not cross the C frame)
                return 1

        def allgather(_ctx, send, recv, n):
            try:
                s = torch.from_numpy(np.ctypeslib.as_array(send, shape=(n,)).copy())
                out = [torch.empty(n, dtype=torch.uint8) for _ in range(world)]
                dist.all_gather(out, s, group=group)
                np.ctypeslib.as_array(recv, shape=(n * world,))[:] = torch.cat(out).numpy()
                return 0
            except Exception:
                return 1

        self._cb = (_abi.ALLREDUCE_FN(allreduce), _abi.ALLGATHER_FN(allgather))
        return _abi.CommOps(None, self._cb[0], self._cb[1])

    @property
    def handle(self):
        return self._h

    def split(self, batch):
        """This rank's input: the whole batch (protocol A) or its keep-all share (B)."""
        if self.protocol == "a" or self.world == 1:
            return batch
        from .resolvers import KeyRangeResolvers

        return KeyRangeResolvers(self.bounds).split(batch, self.rank, keep_all=True)[0]

    def detect_device(self, view, now, new_oldest):
        """view: this rank's batch in device memory (see split); returns the T verdicts."""
        out = np.zeros(max(1, view.txn_count), np.uint8)
        check(self._lib.fdbcs_sharded_detect_device(self._h, C.byref(view), now, new_oldest, out.ctypes.data),
              "fdbcs_sharded_detect_device")
        return out[:view.txn_count]

    def detect_packed(self, batch, now, new_oldest):
        import torch
        from .batch import DeviceBatch

        db = DeviceBatch(self.split(batch), torch.device("cuda", torch.cuda.current_device()))
        return self.detect_device(db.view, now, new_oldest)

    def detect_txns(self, txns, now, new_oldest):
        """The Resolver's per-transaction calls: begin, add per (snapshot, reads, writes), detect."""
        keep = []

        def ranges(rs):
            arr = (_abi.Range * max(1, len(rs)))()
            for i, (b, e) in enumerate(rs):
                bb, eb = C.create_string_buffer(bytes(b), max(1, len(b))), C.create_string_buffer(bytes(e),
                                                                                                   max(1, len(e)))
                keep.append((bb, eb))
                arr[i].begin, arr[i].begin_len = C.cast(bb, C.c_void_p), len(b)
                arr[i].end, arr[i].end_len = C.cast(eb, C.c_void_p), len(e)
            return arr

        check(self._lib.fdbcs_sharded_batch_begin(self._h), "ConflictBatch")
        for snap, reads, writes in txns:
            check(self._lib.fdbcs_sharded_batch_add(self._h, snap, ranges(reads), len(reads), ranges(writes),
                                                    len(writes)), "addTransaction")
        out = np.zeros(max(1, len(txns)), np.uint8)
        check(self._lib.fdbcs_sharded_batch_detect(self._h, now, new_oldest, out.ctypes.data), "detectConflicts")
        return out[:len(txns)]

    def clear(self, v):
        check(self._lib.fdbcs_sharded_clear(self._h, v), "clearConflictSet")

    EXCHANGE_STATS = ("ecap", "retries", "last_max", "shrinks", "ebuf_elems")

    def exchange_stats(self):
        """Protocol B's edge exchange (fdbcs_sharded_exchange_stats)."""
        import ctypes as C
        out = (C.c_int64 * len(self.EXCHANGE_STATS))()
        n = check(self._lib.fdbcs_sharded_exchange_stats(self._h, out, len(out)), "fdbcs_sharded_exchange_stats")
        return dict(zip(self.EXCHANGE_STATS[:n], out[:n]))

    def removal_key_owner(self):
        r = self._lib.fdbcs_sharded_removal_key_owner(self._h)
        if r < -1:
            check(int(r), "fdbcs_sharded_removal_key_owner")
        return int(r)

    def history(self):
        """This rank's part of the history [(key, version)]."""
        return self.local.history()

    def close(self):
        if getattr(self, "_h", None) is not None:
            self.local = None
            self._lib.fdbcs_sharded_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
