"""Python mirror of fdbserver/ConflictSet.h over the HIP C ABI.

Names, argument meaning and error behaviour follow the reference:

  ConflictSet()                 newConflictSet()            ConflictSet.h:28
  cs.clear(v)                   clearConflictSet(cs, v)     ConflictSet.h:29
  cs.close()                    destroyConflictSet(cs)      ConflictSet.h:30
  ConflictBatch(cs)             ConflictBatch::ConflictBatch ConflictSet.h:33
  b.add_transaction(...)        addTransaction              ConflictSet.h:42
  b.detect_conflicts(now, newOldest, nonConflicting, tooOld)
                                detectConflicts             ConflictSet.h:43

``detect_conflicts`` *appends* to the caller's lists, like the reference
(SkipList.cpp:1188-1194).  Errors raise ``FdbcsError`` (the reference's
ASSERT -> internal_error, flow/Error.h:86).
"""
import ctypes as C

import numpy as np

from . import _abi
from ._abi import COMMITTED, CONFLICT, TOO_OLD, FdbcsError, check  # noqa: F401
from .batch import PackedBatch, unpack_history


class ConflictSet:
    def __init__(self, v0=0, device=-1, max_history=0, tail_arena_bytes=0, flags=0):
        self._lib = _abi.lib()
        cfg = _abi.Config(device=device, flags=flags, max_history=max_history, tail_arena_bytes=tail_arena_bytes)
        h = C.c_void_p()
        check(self._lib.fdbcs_create(C.byref(h), v0, C.byref(cfg)), "newConflictSet")
        self._h = h

    @property
    def handle(self):
        if self._h is None:
            raise FdbcsError(_abi.E_STATE, "conflict set destroyed")
        return self._h

    def clear(self, version):
        check(self._lib.fdbcs_clear(self.handle, version), "clearConflictSet")

    set_version = clear

    def close(self):
        if getattr(self, "_h", None) is not None:
            self._lib.fdbcs_destroy(self._h)
            self._h = None

    destroy = close

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # --- introspection ---------------------------------------------------------
    @property
    def oldest_version(self):
        return self._lib.fdbcs_oldest_version(self.handle)

    @property
    def header_version(self):
        return self._lib.fdbcs_header_version(self.handle)

    def history_size(self):
        return check(self._lib.fdbcs_history_size(self.handle), "history_size")

    def removal_key(self):
        n = check(self._lib.fdbcs_removal_key(self.handle, None, 0))
        buf = (C.c_uint8 * max(1, n))()
        self._lib.fdbcs_removal_key(self.handle, buf, n)
        return bytes(buf[:n])

    def dump_arrays(self):
        """(versions, key_len, key_off, key_bytes) numpy arrays of the history."""
        n = self.history_size()
        vers = np.zeros(max(n, 1), np.int64)
        lens = np.zeros(max(n, 1), np.uint32)
        offs = np.zeros(max(n, 1), np.uint64)
        cap = max(64, n * 24)
        while True:
            kb = np.zeros(cap, np.uint8)
            r = self._lib.fdbcs_dump_history(self.handle, n, vers.ctypes.data, lens.ctypes.data, offs.ctypes.data,
                                             kb.ctypes.data, cap)
            if r == _abi.E_CAPACITY:
                cap *= 4
                continue
            check(r, "dump_history")
            return vers[:r], lens[:r], offs[:r], kb

    def history(self):
        """[(key bytes, version), ...] in key order."""
        v, l, o, kb = self.dump_arrays()
        keys, vers = unpack_history(len(v), v, l, o, kb)
        return list(zip(keys, vers))

    def load_history(self, keys, versions, v0=0, oldest=0, removal_key=b""):
        keys = [bytes(k) for k in keys]
        lens = np.array([len(k) for k in keys], np.uint32)
        offs = np.zeros(len(keys), np.uint64)
        if len(keys):
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        blob = np.frombuffer(b"".join(keys) + b"\0", np.uint8).copy()
        vers = np.ascontiguousarray(versions, np.int64)
        rk = np.frombuffer(bytes(removal_key) + b"\0", np.uint8).copy()
        check(self._lib.fdbcs_load_history(self.handle, len(keys), vers.ctypes.data, lens.ctypes.data,
                                           offs.ctypes.data, blob.ctypes.data, v0, oldest, rk.ctypes.data,
                                           len(removal_key)), "load_history")

    def load_history_arrays(self, n, versions, key_len, key_off, key_bytes, v0=0, oldest=0, removal_key=b""):
        rk = np.frombuffer(bytes(removal_key) + b"\0", np.uint8).copy()
        check(self._lib.fdbcs_load_history(self.handle, n, versions.ctypes.data, key_len.ctypes.data,
                                           key_off.ctypes.data, key_bytes.ctypes.data, v0, oldest, rk.ctypes.data,
                                           len(removal_key)), "load_history")

    def enable_stage_timing(self, on=True):
        check(self._lib.fdbcs_enable_stage_timing(self.handle, int(on)))

    def stage_times(self):
        out = (C.c_double * 7)()
        n = self._lib.fdbcs_stage_times(self.handle, out, 7)
        return list(out[:n])

    # --- whole-batch entry points -------------------------------------------------
    STAT_NAMES = ("txns", "reads", "writes", "combined", "pages_merged", "dir_entries", "history", "window_pages",
                  "window_survivors", "dependents", "decision_rounds", "sort_rebucketed", "sort_max_bucket",
                  "tail_arena_bytes", "tail_used", "tail_half", "live_batches", "live_cancelled",
                  "live_timeouts")

    def batch_stats(self):
        """Shape and outcome of the last synchronized batch (fdbcs_batch_stats)."""
        out = (C.c_int64 * len(self.STAT_NAMES))()
        n = check(self._lib.fdbcs_batch_stats(self.handle, out, len(self.STAT_NAMES)))
        return dict(zip(self.STAT_NAMES, [int(x) for x in out[:n]]))

    def detect_packed(self, batch: PackedBatch, now, new_oldest):
        """addTransaction x T + detectConflicts for a packed host batch; returns the verdict bytes."""
        out = np.zeros(max(batch.T, 1), np.uint8)
        check(self._lib.fdbcs_batch_detect_packed(self.handle, C.byref(batch.view()), now, new_oldest,
                                                  out.ctypes.data), "detectConflicts")
        return out[:batch.T]

    def submit_packed(self, batch, now, new_oldest):
        """Pipelined detectConflicts (fdbcs_batch_submit_packed): returns at once;
        the next submit's packing and H2D copy overlap this batch's kernels.
        ``batch``: a PackedBatch or a raw host view (kept alive until wait())."""
        view = batch.view() if hasattr(batch, "view") else batch
        if not hasattr(self, "_inflight"):
            self._inflight = []
        check(self._lib.fdbcs_batch_submit_packed(self.handle, C.byref(view), now, new_oldest), "submit")
        self._inflight.append((batch, view, view.txn_count))

    def wait(self):
        """Verdict bytes of the oldest submitted batch (fdbcs_batch_wait)."""
        _b, _v, T = self._inflight.pop(0)
        out = np.zeros(max(T, 1), np.uint8)
        check(self._lib.fdbcs_batch_wait(self.handle, out.ctypes.data), "wait")
        return out[:T]

    def detect_view(self, host_view, now, new_oldest, out=None):
        """detectConflicts on a raw host fdbcs_batch_view (e.g. generator memory)."""
        T = host_view.txn_count
        if out is None or out.size < max(T, 1):
            out = np.zeros(max(T, 1), np.uint8)
        check(self._lib.fdbcs_batch_detect_packed(self.handle, C.byref(host_view), now, new_oldest,
                                                  out.ctypes.data), "detectConflicts")
        return out[:T]

    def detect_device(self, dev_view, now, new_oldest, dev_verdict_ptr, sync=True):
        """detectConflicts on a batch already resident in device memory."""
        check(self._lib.fdbcs_detect_device(self.handle, C.byref(dev_view), now, new_oldest, dev_verdict_ptr,
                                            int(sync)), "detectConflicts")


class ConflictBatch:
    """``ConflictBatch`` (ConflictSet.h:32-60).  One live batch per conflict set."""

    def __init__(self, cs: ConflictSet):
        self.cs = cs
        self._lib = cs._lib
        check(self._lib.fdbcs_batch_begin(cs.handle), "ConflictBatch")
        self._count = 0
        self._keep = []  # the key buffers (kept to detect_conflicts, as the reference borrows them)

    def add_transaction(self, read_ranges, write_ranges, read_snapshot):
        """read_ranges / write_ranges: sequences of (begin bytes, end bytes)."""
        keep = []

        def ranges(rs):
            arr = (_abi.Range * max(1, len(rs)))()
            for i, (b, e) in enumerate(rs):
                bb, eb = C.create_string_buffer(bytes(b), max(1, len(b))), C.create_string_buffer(bytes(e),
                                                                                                   max(1, len(e)))
                keep.append((bb, eb))
                arr[i].begin = C.cast(bb, C.c_void_p)
                arr[i].begin_len = len(b)
                arr[i].end = C.cast(eb, C.c_void_p)
                arr[i].end_len = len(e)
            return arr

        rs, ws = list(read_ranges), list(write_ranges)
        ra, wa = ranges(rs), ranges(ws)
        keep.append((ra, wa))  # (the range arrays too: a borrowed batch, FDBCS_BORROW_*, reads them at detect)
        check(self._lib.fdbcs_batch_add(self.cs.handle, read_snapshot, ra, len(rs), wa, len(ws)), "addTransaction")
        self._keep.append(keep)
        self._count += 1

    def skip(self, n):
        """n transactions without ranges in one call (fdbcs_batch_skip)."""
        check(self._lib.fdbcs_batch_skip(self.cs.handle, n), "fdbcs_batch_skip")
        self._count += n

    def detect_conflicts(self, now, new_oldest_version, non_conflicting=None, too_old=None):
        """Appends committed indices to ``non_conflicting`` and tooOld indices to
        ``too_old`` (if given); returns the verdict byte array."""
        out = np.zeros(max(self._count, 1), np.uint8)
        try:
            check(self._lib.fdbcs_batch_detect(self.cs.handle, now, new_oldest_version, out.ctypes.data),
                  "detectConflicts")
        finally:
            self._keep = []
        out = out[:self._count]
        if non_conflicting is not None:
            non_conflicting.extend(int(i) for i in np.nonzero(out == COMMITTED)[0])
        if too_old is not None:
            too_old.extend(int(i) for i in np.nonzero(out == TOO_OLD)[0])
        return out
