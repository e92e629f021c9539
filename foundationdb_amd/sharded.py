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

Per batch (the step numbers are SURVEY.md §8e's):

1-2. ``fdbcs_shard_check``: each shard checks every read clipped to its keys.
     valueBefore of a clipped begin is the shard's carry-in.
3.   MAX-reduce of the per-transaction history-conflict flags (T bytes).
4-5. ``fdbcs_shard_apply``: an identical decision and combine on every
     shard, then the shard's part of the merge:
     - a begin node only where the real begin lies;
     - an end node only in the shard holding the end.
6.   Compaction over global boundary indices. The window starts at the first
     boundary >= removalKey anywhere and spans ``3 * |combined| + 10``
     boundaries. Each shard removes in its part, and the "previous node"
     crosses shard edges. The shard holding the window's end supplies the
     new removalKey.
7.   Carry-ins for the next batch: the version of the nearest earlier
     non-empty shard's last boundary, else the global header version v0.

Two exchange back ends share the logic below:

- ``ShardedConflictSet`` runs all shards in one process (on one or several
  devices). Tests use it.
- ``DistShardedConflictSet`` is one shard per rank over torch.distributed:
  RCCL over xGMI, or gloo on CPU.
"""
import ctypes as C
import time

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


KEY_INLINE = 32  # removalKeys up to this length travel inside the compaction all-gather


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

    def __init__(self, lo, hi, device=-1, v0=0, max_history=0):
        self.cs = ConflictSet(v0=v0, device=device, max_history=max_history)
        self._lib = self.cs._lib
        lo_b, hi_b = lo or b"", hi or b""
        check(self._lib.fdbcs_set_shard(self.cs.handle, lo_b, len(lo_b), int(lo is not None), hi_b, len(hi_b),
                                        int(hi is not None)), "set_shard")
        self.lo, self.hi = lo, hi

    def check(self, dev_view, now, new_oldest, dev_hist):
        check(self._lib.fdbcs_shard_check(self.cs.handle, C.byref(dev_view), now, new_oldest, dev_hist), "shard_check")

    def apply(self, dev_view, now, new_oldest, dev_hist, dev_verdict):
        info = (C.c_int64 * 4)()
        check(self._lib.fdbcs_shard_apply(self.cs.handle, C.byref(dev_view), now, new_oldest, dev_hist, dev_verdict,
                                          info), "shard_apply")
        return tuple(info)

    def key_at(self, index):
        n = check(self._lib.fdbcs_shard_key_at(self.cs.handle, index, None, 0), "shard_key_at")
        buf = (C.c_uint8 * max(1, n))()
        self._lib.fdbcs_shard_key_at(self.cs.handle, index, buf, n)
        return bytes(buf[:n])

    def compact(self, part, new_oldest):
        a, b, keep_first, prev = part
        info = (C.c_int64 * 2)()
        check(self._lib.fdbcs_shard_compact(self.cs.handle, a, b, keep_first, prev, new_oldest, info), "shard_compact")
        return tuple(info)

    def finish(self, carry_in, removal_key=None):
        rk = removal_key if removal_key is not None else b""
        check(self._lib.fdbcs_shard_finish(self.cs.handle, carry_in, rk, len(rk), int(removal_key is not None)),
              "shard_finish")

    def clear(self, v):
        self.cs.clear(v)

    def history(self):
        return self.cs.history()

    def removal_key(self):
        return self.cs.removal_key()

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


class ShardedConflictSet:
    """All G shards in this process (on one or several devices): the exchange
    is a device reduction.  ``shard_factory`` builds a shard (tests pass a
    CPU model of the same interface)."""

    def __init__(self, bounds, devices=None, v0=0, max_history=0, shard_factory=Shard):
        import torch

        self.torch = torch
        ranges = _shard_ranges(bounds)
        if devices is None:
            d = torch.cuda.current_device() if torch.cuda.is_available() else -1
            devices = [d] * len(ranges)
        assert len(devices) == len(ranges)
        self.devices = [_device(torch, d) for d in devices]
        self.shards = [shard_factory(lo, hi, device=d, v0=v0, max_history=max_history)
                       for (lo, hi), d in zip(ranges, devices)]
        self.v0 = v0
        self.oldest = 0

    def clear(self, v):
        """clearConflictSet (SkipList.cpp:957-959): every shard empty, carry-ins v."""
        for s in self.shards:
            s.clear(v)
        self.v0 = v

    def detect_device(self, views, now, new_oldest, verdict):
        """views[g]: the batch in shard g's device memory; verdict: uint8 tensor [>= T] on devices[0]."""
        torch = self.torch
        T = views[0].txn_count
        hs = [torch.empty(max(1, T), dtype=torch.uint8, device=d) for d in self.devices]
        for d in set(self.devices):
            _sync(torch, d)
        for s, v, h in zip(self.shards, views, hs):  # steps 1-2
            s.check(v, now, new_oldest, h.data_ptr())
        flags = torch.stack([h.to(self.devices[0]) for h in hs]).amax(0)  # step 3: MAX over shards
        infos, n_comb = [], 0
        for g, (s, v) in enumerate(zip(self.shards, views)):  # steps 4-5
            f = flags.to(self.devices[g])
            out = verdict if g == 0 else torch.empty(max(1, T), dtype=torch.uint8, device=self.devices[g])
            _sync(torch, self.devices[g])
            H, g0, last, n_comb = s.apply(v, now, new_oldest, f.data_ptr(), out.data_ptr())
            infos.append((H, g0, last))
        self._finish(infos, n_comb, new_oldest)

    def detect_packed(self, batch, now, new_oldest):
        """A host PackedBatch through the sharded path; returns the verdict bytes (numpy)."""
        from .batch import DeviceBatch

        staged = {}
        for d in self.devices:
            if d not in staged:
                staged[d] = DeviceBatch(batch, d)
        verdict = self.torch.empty(max(1, batch.T), dtype=self.torch.uint8, device=self.devices[0])
        self.detect_device([staged[d].view for d in self.devices], now, new_oldest, verdict)
        return verdict[:batch.T].cpu().numpy()

    def _finish(self, infos, n_comb, new_oldest):
        rk = None
        if new_oldest > self.oldest:  # step 6
            parts, owner = plan_compaction(infos, n_comb)
            rk = self.shards[owner[0]].key_at(owner[1]) if owner else b""
            hl = [s.compact(p, new_oldest) for s, p in zip(self.shards, parts)]
            self.oldest = new_oldest
        else:
            hl = [(H, last) for H, _g0, last in infos]
        for s, c in zip(self.shards, carry_ins(self.v0, hl)):  # step 7
            s.finish(c, rk)

    @property
    def oldest_version(self):
        return self.oldest

    def history(self):
        out = []
        for s in self.shards:
            out += s.history()
        return out

    def removal_key(self):
        return self.shards[0].removal_key()

    def close(self):
        for s in self.shards:
            s.close()


class DistShardedConflictSet:
    """One shard per torch.distributed rank (RCCL over xGMI on MI355X, gloo on CPU)."""

    def __init__(self, bounds, rank, world, device, v0=0, max_history=0, group=None, shard_factory=Shard):
        import torch
        import torch.distributed as dist

        assert len(bounds) + 1 == world
        self.torch, self.dist, self.group = torch, dist, group
        self.rank, self.world = rank, world
        self.device = _device(torch, device)
        lo, hi = _shard_ranges(bounds)[rank]
        self.shard = shard_factory(lo, hi, device=device, v0=v0, max_history=max_history)
        self.v0 = v0
        self.oldest = 0
        backend = dist.get_backend(group)
        self.coll_dev = self.device if backend == "nccl" else torch.device("cpu")
        self._T = -1
        self.phase_s = None

    def clear(self, v):
        self.shard.clear(v)
        self.v0 = v

    def _buffers(self, T):
        if T != self._T:
            torch = self.torch
            self._h = torch.empty(max(1, T), dtype=torch.uint8, device=self.device)
            self._hc = self._h if self.coll_dev == self.device else torch.empty(max(1, T), dtype=torch.uint8)
            self._T = T
        return self._h, self._hc

    def detect_device(self, view, now, new_oldest, verdict):
        """view: the whole batch in this rank's device memory; verdict: uint8 tensor [>= T] there."""
        torch, dist = self.torch, self.dist
        tick = self._tick
        tick(None)
        h, hc = self._buffers(view.txn_count)
        _sync(torch, self.device)
        self.shard.check(view, now, new_oldest, h.data_ptr())  # steps 1-2 (synchronous)
        tick("check")
        if hc is not h:
            hc.copy_(h)
        dist.all_reduce(hc, op=dist.ReduceOp.MAX, group=self.group)  # step 3
        if hc is not h:
            h.copy_(hc)
        _sync(torch, self.device)  # the engine reads h on its own stream
        tick("flags_allreduce")
        H, g0, last, n_comb = self.shard.apply(view, now, new_oldest, h.data_ptr(), verdict.data_ptr())  # 4-5
        tick("apply")
        infos = self._allgather([H, g0, last])
        tick("allgather1")
        rk = None
        if new_oldest > self.oldest:  # step 6
            parts, owner = plan_compaction([tuple(x) for x in infos], n_comb)
            # the owner reads the new removalKey before its compaction moves the indices
            key = self.shard.key_at(owner[1]) if owner is not None and owner[0] == self.rank else b""
            tick("key_at")
            Hn, lastn = self.shard.compact(parts[self.rank], new_oldest)
            tick("compact")
            # one all-gather carries (H, last version) for the carry-ins and a short removalKey
            inline = key if len(key) <= KEY_INLINE else b""
            words = [Hn, lastn, len(key)] + _pack_key(inline)
            got = self._allgather(words)
            tick("allgather2")
            hl = [(x[0], x[1]) for x in got]
            if owner is None:
                rk = b""  # the scan reached the end: removalKey wraps
            elif got[owner[0]][2] <= KEY_INLINE:
                rk = _unpack_key(got[owner[0]][3:], got[owner[0]][2])
            else:
                rk = self._broadcast_key(owner, key)
            self.oldest = new_oldest
        else:
            hl = [(x[0], x[2]) for x in infos]
        self.shard.finish(carry_ins(self.v0, hl)[self.rank], rk)  # step 7
        tick("finish")

    def enable_phase_timing(self, on=True):
        """Accumulate host wall time per protocol phase (``phase_times``)."""
        self.phase_s = {} if on else None

    def _tick(self, name):
        if self.phase_s is None:
            return
        t = time.perf_counter()
        if name is not None:
            self.phase_s[name] = self.phase_s.get(name, 0.0) + t - self._t
        self._t = t

    def detect_packed(self, batch, now, new_oldest):
        from .batch import DeviceBatch

        db = DeviceBatch(batch, self.device)
        verdict = self.torch.empty(max(1, batch.T), dtype=self.torch.uint8, device=self.device)
        self.detect_device(db.view, now, new_oldest, verdict)
        return verdict[:batch.T].cpu().numpy()

    def _broadcast_key(self, owner, key):
        """A removalKey too long for the all-gather, from the shard that read it."""
        torch, dist = self.torch, self.dist
        buf = torch.zeros(_abi.MAX_KEY + 4, dtype=torch.uint8)
        if owner[0] == self.rank:
            buf[:4 + len(key)] = torch.frombuffer(bytearray(len(key).to_bytes(4, "little") + key), dtype=torch.uint8)
        buf = buf.to(self.coll_dev)
        dist.broadcast(buf, src=owner[0], group=self.group)
        raw = buf.cpu().numpy()
        n = int.from_bytes(raw[:4].tobytes(), "little")
        return raw[4:4 + n].tobytes()

    def _allgather(self, vals):
        torch, dist = self.torch, self.dist
        t = torch.tensor(vals, dtype=torch.int64, device=self.coll_dev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [o.cpu().tolist() for o in out]

    @property
    def oldest_version(self):
        return self.oldest

    def history(self):
        return self.shard.history()

    def removal_key(self):
        return self.shard.removal_key()

    def close(self):
        self.shard.close()
