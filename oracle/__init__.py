"""Oracles for the Resolver conflict set -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this package, and only as the checker / reported CPU baseline.  The product
(foundationdb_amd) never imports it.

  spec.SpecConflictSet / SpecBatch   naive pure-Python restatement (small cases)
  CpuSpec                            C++ restatement (oracle/cpu_spec.cpp), fast

Parity status: UNPINNED by execution of the reference -- see spec.py's header.
"""
import ctypes as C
import os

import numpy as np

from .spec import COMMITTED, CONFLICT, TOO_OLD, SpecBatch, SpecConflictSet  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_spec.so")

_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `python -m foundationdb_amd.build`")
        L = C.CDLL(LIB_PATH)
        L.orc_create.restype = C.c_void_p
        L.orc_create.argtypes = [C.c_int64]
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_clear.argtypes = [C.c_void_p, C.c_int64]
        L.orc_size.restype = C.c_int64
        L.orc_size.argtypes = [C.c_void_p]
        L.orc_v0.restype = C.c_int64
        L.orc_v0.argtypes = [C.c_void_p]
        L.orc_oldest.restype = C.c_int64
        L.orc_oldest.argtypes = [C.c_void_p]
        L.orc_removal_key.restype = C.c_int32
        L.orc_removal_key.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.orc_detect.restype = C.c_int
        L.orc_detect.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]
        L.orc_dump.restype = C.c_int64
        L.orc_dump.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.orc_load.restype = C.c_int
        L.orc_load.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                               C.c_int64, C.c_void_p, C.c_uint32]
        _lib = L
    return _lib


class CpuSpec:
    """C++ oracle with the same whole-batch interface as foundationdb_amd.ConflictSet."""

    def __init__(self, v0=0):
        self._l = _load()
        self._h = C.c_void_p(self._l.orc_create(v0))

    def close(self):
        if self._h:
            self._l.orc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def clear(self, v):
        self._l.orc_clear(self._h, v)

    def detect_packed(self, batch, now, new_oldest):
        out = np.zeros(max(batch.T, 1), np.uint8)
        r = self._l.orc_detect(self._h, C.byref(batch.view()), now, new_oldest, out.ctypes.data)
        if r != 0:
            raise RuntimeError(f"oracle status {r}")
        return out[:batch.T]

    def history_size(self):
        return self._l.orc_size(self._h)

    @property
    def oldest_version(self):
        return self._l.orc_oldest(self._h)

    @property
    def header_version(self):
        return self._l.orc_v0(self._h)

    def removal_key(self):
        n = self._l.orc_removal_key(self._h, None, 0)
        buf = (C.c_uint8 * max(1, n))()
        self._l.orc_removal_key(self._h, buf, n)
        return bytes(buf[:n])

    def dump_arrays(self):
        n = self.history_size()
        vers = np.zeros(max(n, 1), np.int64)
        lens = np.zeros(max(n, 1), np.uint32)
        offs = np.zeros(max(n, 1), np.uint64)
        cap = max(64, n * 24)
        while True:
            kb = np.zeros(cap, np.uint8)
            r = self._l.orc_dump(self._h, n, vers.ctypes.data, lens.ctypes.data, offs.ctypes.data, kb.ctypes.data,
                                 cap)
            if r == -8:
                cap *= 4
                continue
            return vers[:r], lens[:r], offs[:r], kb

    def history(self):
        v, l, o, kb = self.dump_arrays()
        return [(kb[int(o[i]):int(o[i]) + int(l[i])].tobytes(), int(v[i])) for i in range(len(v))]

    def load_history_arrays(self, n, versions, key_len, key_off, key_bytes, v0=0, oldest=0, removal_key=b""):
        rk = np.frombuffer(bytes(removal_key) + b"\0", np.uint8).copy()
        self._l.orc_load(self._h, n, versions.ctypes.data, key_len.ctypes.data, key_off.ctypes.data,
                         key_bytes.ctypes.data, v0, oldest, rk.ctypes.data, len(removal_key))


def spec_detect(cs, batch, now, new_oldest):
    """Run one PackedBatch through the pure-Python spec; returns the verdict list."""
    b = SpecBatch(cs)
    for snap, reads, writes in batch.txns():
        b.add_transaction(reads, writes, snap)
    verdict, _nc, _to = b.detect_conflicts(now, new_oldest)
    return verdict
