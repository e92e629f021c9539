"""Synthetic Resolver batches from the native generator."""
import ctypes as C

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

    def close(self):
        if getattr(self, "_g", None):
            self._lib.fdbwl_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
