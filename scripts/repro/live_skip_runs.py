"""Repro of tests/test_gpu_parity.py::test_per_transaction_skip_runs with live
ingest: at the first verdict mismatch, the device batch view the live kernel
built (fdbcs_last_device_batch) against the packed batch's, entry by entry.

usage: python scripts/repro/live_skip_runs.py
"""
import ctypes as C
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from gen import mixed_stream  # noqa: E402
from foundationdb_amd import ConflictBatch, ConflictSet, _abi  # noqa: E402
from foundationdb_amd.batch import PackedBatch  # noqa: E402
from oracle import CpuSpec  # noqa: E402


def dev_array(ptr, n, dtype):
    import torch
    t = torch.empty(max(n, 1), dtype={np.int64: torch.int64, np.int32: torch.int32, np.uint64: torch.int64,
                                      np.uint32: torch.int32}[dtype], device="cuda")
    if n:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(n * t.element_size()), 3)
        hip.hipDeviceSynchronize()
    return t.cpu().numpy()[:n].view(dtype)


def main():
    import torch
    torch.cuda.set_device(0)
    cs = ConflictSet(device=0)
    for seed in range(3):
        cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
        c = CpuSpec()
        rng = random.Random(seed)
        for bi, (batch, now, nold) in enumerate(mixed_stream(seed, n_batches=8, max_txns=400, keyspace=3000)):
            txns = []
            for t in batch.txns():
                if rng.random() < 0.3:
                    txns += [(rng.randrange(0, now), [], [])] * rng.randint(1, 5)
                txns.append(t)
            txns += [(0, [], [])] * rng.randint(0, 3)
            pb = PackedBatch.from_txns(txns)
            vc = c.detect_packed(pb, now, nold)
            b = ConflictBatch(cs)
            pending = 0
            for snap, r, w in txns:
                if not r and not w:
                    pending += 1
                    continue
                if pending:
                    b.skip(pending)
                    pending = 0
                b.add_transaction(r, w, snap)
            if pending:
                b.skip(pending)
            v = b.detect_conflicts(now, nold)
            st = cs.batch_stats()
            print(f"seed {seed} batch {bi}: T={pb.T} R={pb.R} W={pb.W} live={st['live_batches']} "
                  f"cancelled={st['live_cancelled']} same={np.array_equal(v, vc)}", flush=True)
            if not np.array_equal(v, vc):
                bad = np.nonzero(v != vc)[0]
                print("  mismatched txns:", bad.tolist(), "gpu", v[bad].tolist(), "cpu", vc[bad].tolist())
                dv = _abi.BatchView()
                r = cs._lib.fdbcs_last_device_batch(cs.handle, C.byref(dv))
                print("  last_device_batch:", r, dv.txn_count, dv.read_count, dv.write_count)
                if r == 0:
                    T, R, W = dv.txn_count, dv.read_count, dv.write_count
                    snap = dev_array(dv.snapshot, T, np.int64)
                    ro = dev_array(dv.read_off, T + 1, np.int32)
                    wo = dev_array(dv.write_off, T + 1, np.int32)
                    klen = dev_array(dv.key_len, 2 * (R + W), np.uint32)
                    print("  snap same:", np.array_equal(snap, pb.snapshot), "ro same:",
                          np.array_equal(ro, pb.read_off.astype(np.int32)), "wo same:",
                          np.array_equal(wo, pb.write_off.astype(np.int32)), "klen same:",
                          np.array_equal(klen, pb.key_len))
                    for t in bad[:3]:
                        print("   txn", t, txns[t], "dev snap", snap[t], "ro", ro[t], ro[t + 1], "wo", wo[t], wo[t + 1])
                return
    cs.close()


if __name__ == "__main__":
    main()
