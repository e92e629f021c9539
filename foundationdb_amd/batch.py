"""Packed batch layout shared by the C ABI, the generators and the oracle.

``PackedBatch`` holds a whole ConflictBatch in the structure-of-arrays form of
``fdbcs_batch_view`` (include/fdbcs.h): every transaction's reads occupy key
slots first (begin 2r, end 2r+1), then every write (2R+2w, 2R+2w+1).
"""
import ctypes as C

import numpy as np

from ._abi import BatchView


def _ptr(a):
    return a.ctypes.data if a.size else None


class PackedBatch:
    def __init__(self, snapshot, read_off, write_off, key_off, key_len, key_bytes):
        self.snapshot = np.ascontiguousarray(snapshot, dtype=np.int64)
        self.read_off = np.ascontiguousarray(read_off, dtype=np.int32)
        self.write_off = np.ascontiguousarray(write_off, dtype=np.int32)
        self.key_off = np.ascontiguousarray(key_off, dtype=np.uint64)
        self.key_len = np.ascontiguousarray(key_len, dtype=np.uint32)
        self.key_bytes = np.ascontiguousarray(key_bytes, dtype=np.uint8)
        self.T = int(self.snapshot.size)
        self.R = int(self.read_off[-1]) if self.read_off.size else 0
        self.W = int(self.write_off[-1]) if self.write_off.size else 0
        self._view = None

    @classmethod
    def from_txns(cls, txns):
        """txns: iterable of (read_snapshot, [(begin, end), ...] reads, [...] writes)."""
        txns = list(txns)
        snaps, roff, woff = [], [0], [0]
        rkeys, wkeys = [], []
        for snap, reads, writes in txns:
            snaps.append(snap)
            for b, e in reads:
                rkeys += [bytes(b), bytes(e)]
            for b, e in writes:
                wkeys += [bytes(b), bytes(e)]
            roff.append(roff[-1] + len(reads))
            woff.append(woff[-1] + len(writes))
        keys = rkeys + wkeys
        lens = np.array([len(k) for k in keys], dtype=np.uint32)
        offs = np.zeros(len(keys), dtype=np.uint64)
        if len(keys):
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        blob = np.frombuffer(b"".join(keys), dtype=np.uint8) if keys else np.zeros(0, np.uint8)
        return cls(np.array(snaps, dtype=np.int64), np.array(roff), np.array(woff), offs, lens, blob.copy())

    @classmethod
    def from_view(cls, v):
        """Copy a generator-owned fdbcs_batch_view into numpy arrays."""
        T, R, W = v.txn_count, v.read_count, v.write_count
        slots = 2 * (R + W)

        def arr(ptr, ctype, n, dtype):
            if n == 0:
                return np.zeros(0, dtype)
            return np.ctypeslib.as_array((ctype * n).from_address(ptr)).astype(dtype, copy=True)

        return cls(arr(v.snapshot, C.c_int64, T, np.int64), arr(v.read_off, C.c_int32, T + 1, np.int32),
                   arr(v.write_off, C.c_int32, T + 1, np.int32), arr(v.key_off, C.c_uint64, slots, np.uint64),
                   arr(v.key_len, C.c_uint32, slots, np.uint32),
                   arr(v.key_bytes, C.c_uint8, int(v.key_bytes_len), np.uint8))

    def nbytes(self):
        """Host bytes of the batch (what crosses PCIe in one staged transfer)."""
        return sum(a.nbytes for a in (self.snapshot, self.read_off, self.write_off, self.key_off, self.key_len,
                                      self.key_bytes))

    def view(self):
        if self._view is None:
            v = BatchView()
            v.txn_count, v.read_count, v.write_count = self.T, self.R, self.W
            v.snapshot = _ptr(self.snapshot)
            v.read_off = _ptr(self.read_off)
            v.write_off = _ptr(self.write_off)
            v.key_off = _ptr(self.key_off)
            v.key_len = _ptr(self.key_len)
            v.key_bytes = _ptr(self.key_bytes)
            v.key_bytes_len = int(self.key_bytes.size)
            self._view = v
        return self._view

    def key(self, slot):
        o, n = int(self.key_off[slot]), int(self.key_len[slot])
        return self.key_bytes[o:o + n].tobytes()

    def txns(self):
        """Back to (snapshot, reads, writes) tuples (for the pure-Python spec)."""
        out = []
        for t in range(self.T):
            reads = [(self.key(2 * r), self.key(2 * r + 1)) for r in range(self.read_off[t], self.read_off[t + 1])]
            writes = [(self.key(2 * self.R + 2 * w), self.key(2 * self.R + 2 * w + 1))
                      for w in range(self.write_off[t], self.write_off[t + 1])]
            out.append((int(self.snapshot[t]), reads, writes))
        return out


def unpack_history(n, versions, key_len, key_off, key_bytes):
    """(keys list, versions list) from dump arrays."""
    keys = [key_bytes[int(key_off[i]):int(key_off[i]) + int(key_len[i])].tobytes() for i in range(n)]
    return keys, [int(v) for v in versions[:n]]


class DeviceBatch:
    """A batch staged in device memory: the tensors plus the ``fdbcs_batch_view``
    over them (the input of ``fdbcs_detect_device`` and the sharded entry points).

    ``src`` is a ``PackedBatch`` or a host ``BatchView``; ``device`` a torch device.
    """

    def __init__(self, src, device):
        import torch

        v = src.view() if isinstance(src, PackedBatch) else src
        T, R, W = v.txn_count, v.read_count, v.write_count
        slots = 2 * (R + W)

        def arr(ptr, ctype, n, dtype):
            if n == 0:
                return torch.zeros(1, dtype=torch.uint8, device=device)
            a = np.ctypeslib.as_array((ctype * n).from_address(ptr)).astype(dtype, copy=True)
            return torch.from_numpy(a).to(device)

        self.tensors = [arr(v.snapshot, C.c_int64, T, np.int64), arr(v.read_off, C.c_int32, T + 1, np.int32),
                        arr(v.write_off, C.c_int32, T + 1, np.int32), arr(v.key_off, C.c_uint64, slots, np.int64),
                        arr(v.key_len, C.c_uint32, slots, np.int32),
                        arr(v.key_bytes, C.c_uint8, int(v.key_bytes_len), np.uint8)]
        dv = BatchView()
        dv.txn_count, dv.read_count, dv.write_count = T, R, W
        t = self.tensors
        dv.snapshot, dv.read_off, dv.write_off = t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr()
        dv.key_off, dv.key_len, dv.key_bytes = t[3].data_ptr(), t[4].data_ptr(), t[5].data_ptr()
        dv.key_bytes_len = int(v.key_bytes_len)
        self.view = dv
        self.T = T
        if self.tensors[0].is_cuda:
            torch.cuda.synchronize(self.tensors[0].device)  # the engines read it on their own streams
