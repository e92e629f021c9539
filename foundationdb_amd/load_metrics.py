"""Resolver load metrics: the Resolver's ``iopsSample``.

Mirrors ``TransientStorageMetricSample`` (fdbserver/StorageMetrics.actor.h:98-182)
as the Resolver uses it (fdbserver/Resolver.actor.cpp:47,65,146-151,276-289):

  * ``add_batch``       -- the per-range ``addAndExpire`` loop of one batch
                           (:146-151), rolled on the device over the batch
                           already resident in HBM;
  * ``poll``            -- ``iopsSample.poll()`` every SAMPLE_POLL_TIME (:286-289);
  * ``get_estimate``    -- ResolutionMetricsRequest (:276-277);
  * ``split_estimate``  -- ResolutionSplitRequest (:279-283), with ``used`` as
                           the Resolver computes it.

Knob defaults are fdbserver/Knobs.cpp:269,278-280.  The sample itself is host
state (the reference's IndexedSet); only the roll runs on the GPU.  Every call
goes through libfdbcs.so (include/fdbcs.h); there is no Python fallback.
"""
import ctypes as C

from . import _abi

KEY_BYTES_PER_SAMPLE = 20000   # Knobs.cpp:269
SAMPLE_OFFSET_PER_KEY = 100    # Knobs.cpp:278
SAMPLE_EXPIRATION_TIME = 1.0   # Knobs.cpp:279
SAMPLE_POLL_TIME = 0.1         # Knobs.cpp:280
ALL_KEYS = (b"", b"\xff\xff")  # allKeys (fdbclient/SystemData.cpp)


class IopsSample:
    """A TransientStorageMetricSample whose per-batch roll runs on the GPU."""

    def __init__(self, units_per_sample=KEY_BYTES_PER_SAMPLE, seed=0):
        self._lib = _abi.lib()
        h = C.c_void_p()
        _abi.check(self._lib.fdbcs_sample_create(C.byref(h), int(units_per_sample), int(seed) & (2**64 - 1)),
                   "fdbcs_sample_create")
        self._h = h
        self.units = int(units_per_sample)

    def close(self):
        if self._h is not None and self._h.value:
            self._lib.fdbcs_sample_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_batch(self, cs, expiration, dev_batch=None, offset_per_key=SAMPLE_OFFSET_PER_KEY):
        """Resolver.actor.cpp:146-151 for one batch.  ``cs`` is the
        ConflictSet that resolved it; ``dev_batch`` a device-resident
        BatchView (None: the batch ``cs`` resolved last from host memory).
        Returns the number of keys sampled."""
        n = C.c_int64()
        view = C.byref(dev_batch) if dev_batch is not None else None
        _abi.check(self._lib.fdbcs_sample_add_batch(self._h, cs.handle, view, int(offset_per_key),
                                                    float(expiration), C.byref(n)), "fdbcs_sample_add_batch")
        return n.value

    def attach(self, cs, offset_per_key=SAMPLE_OFFSET_PER_KEY):
        """fdbcs_sample_attach: ``cs``'s per-transaction ingest rolls every
        batch for this sample on the device (None: detach); ``add_batch(cs,
        ...)`` after ``detect_conflicts`` then only inserts the entries."""
        _abi.check(self._lib.fdbcs_sample_attach(self._h, cs.handle if cs is not None else None,
                                                 int(offset_per_key)), "fdbcs_sample_attach")

    def add_metric(self, key: bytes, metric: int):
        _abi.check(self._lib.fdbcs_sample_add_metric(self._h, key, len(key), int(metric)), "fdbcs_sample_add_metric")

    def poll(self, now):
        _abi.check(self._lib.fdbcs_sample_poll(self._h, float(now)), "fdbcs_sample_poll")

    def get_estimate(self, begin: bytes = ALL_KEYS[0], end: bytes = ALL_KEYS[1]) -> int:
        return _abi.check(self._lib.fdbcs_sample_estimate(self._h, begin, len(begin), end, len(end)),
                          "fdbcs_sample_estimate")

    def split_estimate(self, begin: bytes, end: bytes, offset: int, front: bool = True) -> bytes:
        # the split key is a prefix of a sampled key or of begin / end
        for cap in (max(len(begin), len(end)) + 64, _abi.MAX_KEY):
            buf = C.create_string_buffer(cap)
            n = self._lib.fdbcs_sample_split(self._h, begin, len(begin), end, len(end), int(offset),
                                             1 if front else 0, buf, len(buf))
            if n != _abi.E_CAPACITY:
                break
        _abi.check(n, "fdbcs_sample_split")
        return buf.raw[:n]

    def resolution_split(self, begin: bytes, end: bytes, offset: int, front: bool):
        """ResolutionSplitReply {key, used} (Resolver.actor.cpp:279-283)."""
        key = self.split_estimate(begin, end, offset, front)
        used = self.get_estimate(begin, key) if front else self.get_estimate(key, end)
        return key, used

    def size(self) -> int:
        return self._lib.fdbcs_sample_size(self._h)

    def queue_size(self) -> int:
        return self._lib.fdbcs_sample_queue_size(self._h)

    def items(self):
        """[(key, metric)] in key order."""
        out = []
        m = C.c_int64()
        buf = C.create_string_buffer(_abi.MAX_KEY)
        for i in range(self.size()):
            ln = _abi.check(self._lib.fdbcs_sample_entry(self._h, i, buf, len(buf), C.byref(m)), "fdbcs_sample_entry")
            out.append((buf.raw[:ln], m.value))
        return out
