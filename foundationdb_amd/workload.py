"""Synthetic Resolver batches from the native generator."""
import ctypes as C

import numpy as np

from . import _abi
from .batch import PackedBatch


class Workload:
    def __init__(self, config, txns=0, threads=0):
        self._lib = _abi.workload_lib()
        self._g = self._lib.fdbwl_create(config, txns, threads)
        if not self._g:
            raise ValueError(f"unknown workload config {config}")
        self.config = config

    def view(self, index):
        """(fdbcs_batch_view into generator memory, now, new_oldest); valid until the next call."""
        v = _abi.BatchView()
        now, nold = C.c_int64(), C.c_int64()
        _abi.check(self._lib.fdbwl_generate(self._g, index, C.byref(v), C.byref(now), C.byref(nold)), "generate")
        return v, now.value, nold.value

    def batch(self, index):
        v, now, nold = self.view(index)
        return PackedBatch.from_view(v), now, nold

    def set_successor(self, source):
        """Config 4: the wide read ends at the S-th boundary after its begin in
        ``source``'s current history -- a ConflictSet (the
        engine's fdbcs_nth_after) or an oracle CpuSpec (orc_nth_after); None
        restores the log-uniform key-space fraction."""
        if source is None:
            self._lib.fdbwl_set_successor(self._g, None, None)
            return
        if hasattr(source, "_l"):  # oracle.CpuSpec
            fn = C.cast(source._l.orc_nth_after, C.c_void_p)
            ctx = source._h
        else:
            fn = C.cast(self._lib.fdbwl_succ_engine, C.c_void_p)
            ctx = source.handle
        self._succ_keep = source
        self._lib.fdbwl_set_successor(self._g, fn, ctx)

    def prefill(self, cs, first, n):
        """Grow cs's history through batches [first, first + n) (native, pipelined)."""
        _abi.check(self._lib.fdbwl_prefill(self._g, cs.handle, first, n), "prefill")

    def prepare_run(self, first, n, split=None):
        """Batches [first, first + n) pre-generated in the Resolver's per-transaction form.
        split = (bounds, rank): each batch reduced to that rank's protocol-B
        share (fdbwl_run_prepare_split)."""
        return ResolverRun(self, first, n, split)

    def close(self):
        if getattr(self, "_g", None):
            self._lib.fdbwl_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ResolverRun:
    """Prepared batches driven through the Resolver's loop in native code
    (Resolver.actor.cpp:140-153: ConflictBatch, T x addTransaction,
    detectConflicts), so the timed window holds no Python."""

    def __init__(self, wl, first, n, split=None):
        self._lib = wl._lib
        if split is None:
            self._r = self._lib.fdbwl_run_prepare(wl._g, first, n)
        else:
            bounds, rank = split
            kb = np.frombuffer(b"".join(bounds) + b"\0", np.uint8).copy()
            offs = np.array(np.cumsum([0] + [len(b) for b in bounds])[:-1] if bounds else [0], np.uint64)
            lens = np.array([len(b) for b in bounds] or [0], np.uint32)
            self._r = self._lib.fdbwl_run_prepare_split(wl._g, first, n, len(bounds) + 1, kb.ctypes.data,
                                                        offs.ctypes.data, lens.ctypes.data, rank)
        if not self._r:
            raise RuntimeError("fdbwl_run_prepare failed")
        self.n = n
        self.T = self._lib.fdbwl_run_txns(self._r)

    def run(self, cs, verdicts=True, sample=None, expire0=1.0, expire_step=0.01):
        """Runs every batch; returns (per-batch window in us, its addTransaction
        part in us, verdicts n x T or None).  cs: a ConflictSet, or a
        sharded.ShardedResolver (this rank's fdbcs_sharded calls).  sample: a
        load_metrics.IopsSample -- each window then ends with the batch's
        iopsSample adds (resolverCount > 1, Resolver.actor.cpp:146-151)."""
        us = np.zeros(max(self.n, 1), np.float64)
        add = np.zeros(max(self.n, 1), np.float64)
        out = np.zeros((max(self.n, 1), max(self.T, 1)), np.uint8) if verdicts else None
        optr = out.ctypes.data if verdicts else None
        if sample is not None:
            from .load_metrics import SAMPLE_OFFSET_PER_KEY
            _abi.check(self._lib.fdbwl_run_resolver_sampled(self._r, cs.handle, sample._h, SAMPLE_OFFSET_PER_KEY,
                                                            float(expire0), float(expire_step), us.ctypes.data,
                                                            add.ctypes.data, optr), "resolver loop (sampled)")
        else:
            fn = self._lib.fdbwl_run_resolver_sharded if getattr(cs, "sharded", False) else self._lib.fdbwl_run_resolver
            _abi.check(fn(self._r, cs.handle, us.ctypes.data, add.ctypes.data, optr), "resolver loop")
        return us[:self.n], add[:self.n], (out[:self.n, :self.T] if verdicts else None)

    def key_bytes(self, i=0):
        """Key bytes of prepared batch i (SURVEY.md §8d's input term)."""
        return int(self._lib.fdbwl_run_key_bytes(self._r, i))

    def close(self):
        if getattr(self, "_r", None):
            self._lib.fdbwl_run_destroy(self._r)
            self._r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
