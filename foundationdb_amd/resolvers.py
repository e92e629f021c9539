"""Key-range resolvers: FoundationDB's multi-resolver scale-out, one conflict set per GPU.

The reference scales the Resolver out by key range: the master assigns each
resolver a key range (masterserver.actor.cpp:964-1020), the proxy sends each
resolver the transactions whose read or write ranges intersect its keys, with
those ranges unclipped (ResolutionRequestBuilder, MasterProxyServer.actor.cpp:
242-320), every resolver runs its own ConflictSet on that sub-batch, and the
proxy takes the per-transaction minimum of the verdicts (:558-569).

Here resolver g is the conflict set on GPU g.  ``KeyRangeResolvers.split``
is the proxy's split (native: ``fdbcs_split_batch``); the combine is
``fdbcs_scatter_verdicts`` into a T-byte array prefilled with
TransactionCommitted followed by a MIN all-reduce (RCCL over xGMI; gloo on
CPU) -- the element-wise minimum is exactly the proxy's loop.
"""
import ctypes as C

import numpy as np

from . import _abi
from .batch import PackedBatch
from ._abi import check


def uniform_bounds(nres, width=8):
    """nres-1 bounds cutting the key space into equal slices of its first `width` bytes."""
    return [((g << (8 * width)) // nres).to_bytes(width, "big") for g in range(1, nres)]


class KeyRangeResolvers:
    """A static key -> resolver map: resolver g owns [bounds[g-1], bounds[g])."""

    def __init__(self, bounds):
        self.bounds = [bytes(b) for b in bounds]
        if any(a >= b for a, b in zip(self.bounds, self.bounds[1:])):
            raise ValueError("resolver bounds must ascend strictly")
        self.n = len(self.bounds) + 1
        lens = np.array([len(b) for b in self.bounds] or [0], np.uint32)
        offs = np.zeros(max(1, len(self.bounds)), np.uint64)
        if len(self.bounds) > 1:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        self._blob = np.frombuffer(b"".join(self.bounds) + b"\0", np.uint8).copy()
        self._lens, self._offs = lens, offs
        self._lib = _abi.lib()

    def owner(self, key):
        k = np.frombuffer(bytes(key) + b"\0", np.uint8)
        return check(self._lib.fdbcs_key_owner(self.n, self._blob.ctypes.data, self._offs.ctypes.data,
                                               self._lens.ctypes.data, k.ctypes.data, len(key)), "key_owner")

    def split(self, batch: PackedBatch, g, keep_all=False):
        """(sub-batch PackedBatch, txn_index int32 array) that resolver g receives.
        keep_all: every transaction stays (with only its ranges intersecting g's
        keys) -- the per-shard input of the exact sharded protocol B."""
        T, R, W = batch.T, batch.R, batch.W
        slots = 2 * (R + W)
        snap = np.zeros(max(T, 1), np.int64)
        roff = np.zeros(T + 1, np.int32)
        woff = np.zeros(T + 1, np.int32)
        koff = np.zeros(max(slots, 1), np.uint64)
        klen = np.zeros(max(slots, 1), np.uint32)
        idx = np.zeros(max(T, 1), np.int32)
        out = _abi.BatchView()
        fn = self._lib.fdbcs_split_batch_keep_all if keep_all else self._lib.fdbcs_split_batch
        check(fn(C.byref(batch.view()), self.n, self._blob.ctypes.data,
                                          self._offs.ctypes.data, self._lens.ctypes.data, g, C.byref(out),
                                          snap.ctypes.data, roff.ctypes.data, woff.ctypes.data, koff.ctypes.data,
                                          klen.ctypes.data, idx.ctypes.data), "split_batch")
        t, r, w = out.txn_count, out.read_count, out.write_count
        sub = PackedBatch(snap[:t], roff[:t + 1], woff[:t + 1], koff[:2 * (r + w)], klen[:2 * (r + w)],
                          batch.key_bytes)
        return sub, idx[:t].copy()


def scatter_verdicts(cs, dev_sub, dev_index, n, dev_global):
    """One resolver's share of the combine on the GPU (device pointers, ints).
    cs: the resolver's ConflictSet (its stream) or None (null stream)."""
    lib = _abi.lib()
    check(lib.fdbcs_scatter_verdicts(cs.handle if cs is not None else None, dev_sub, dev_index, n, dev_global),
          "scatter_verdicts")


def combine(T, parts):
    """Host form of the proxy's combine: parts = [(sub_verdicts, txn_index), ...]."""
    out = np.full(T, _abi.COMMITTED, np.uint8)
    for v, idx in parts:
        np.minimum.at(out, idx, np.asarray(v, np.uint8))
    return out
