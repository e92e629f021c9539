"""Per-batch window / add times of the Resolver loop with live ingest, in runs
of `per_run` batches (the bench's latency leg shape), with the live counters
(fdbcs_batch_stats [16], [17]) after each run.

usage: python scripts/diag_live.py [runs=5] [per_run=100] [prefill=300] [pin]
"""
import sys
import time

import numpy as np


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    prefill = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    pin = len(sys.argv) > 4 and sys.argv[4] == "pin"
    import torch
    torch.cuda.set_device(0)
    if pin:  # (the bench's host-thread placement)
        import bench
        print("affinity:", bench.pin_host(0), flush=True)
    from foundationdb_amd import ConflictSet
    from foundationdb_amd.workload import Workload
    wl = Workload(2, txns=5000)
    cs = ConflictSet(device=0)
    wl.prefill(cs, 0, prefill - 50)
    r = wl.prepare_run(prefill - 50, 50)
    r.run(cs, verdicts=False)
    nxt = prefill
    import ctypes as C
    buf = (C.c_int64 * 32)()
    phases = buf if cs._lib.fdbcs_debug_phases(cs.handle, buf, 32) > 0 else None
    for k in range(runs):
        t = time.time()
        r = wl.prepare_run(nxt, per)
        gen_s = time.time() - t
        if phases is not None:  # (FDBCS_PHASES build: batch by batch, the live kernel's clock points)
            us, add = np.zeros(per), np.zeros(per)
            ph = []
            for j in range(per):
                r1 = wl.prepare_run(nxt + j, 1)
                u, a_, _ = r1.run(cs, verdicts=False)
                us[j], add[j] = u[0], a_[0]
                cs._lib.fdbcs_debug_phases(cs.handle, phases, 32)
                p = np.array(phases[:32], np.int64)
                # final seen -> last wave out, last wave out -> k_ss_guard's start, poller start -> final seen;
                # the last group: final -> its start, its acquire, toff + window, its ranges
                ph.append(((p[11] - p[10]) * 0.01, (p[12] - p[11]) * 0.01, (p[10] - p[13]) * 0.01,
                           (p[20] - p[10]) * 0.01, (p[21] - p[20]) * 0.01, (p[22] - p[21]) * 0.01,
                           (p[23] - p[22]) * 0.01, (p[11] - p[23]) * 0.01,
                           (p[14] - p[22]) * 0.01, (p[15] - p[14]) * 0.01, (p[23] - p[15]) * 0.01))
            ph = np.array(ph)
            m = ph.mean(axis=0)
            print(f"   live phases (us, mean): final->last wave out {m[0]:.1f}, last wave out->guard start "
                  f"{m[1]:.1f}, kernel start->final {m[2]:.1f}; last group: final->start {m[3]:.1f}, acquire "
                  f"{m[4]:.1f}, toff+window {m[5]:.1f}, ranges {m[6]:.1f} (headers {m[8]:.1f}, range issue "
                  f"{m[9]:.1f}, store drain {m[10]:.1f}), end->last wave out {m[7]:.1f}")
        else:
            us, add, _ = r.run(cs, verdicts=False)
        nxt += per
        st = cs.batch_stats()
        slow = np.nonzero(us > 400)[0]
        print(f"run {k}: gen {gen_s:.2f}s  window p50 {np.median(us):.1f} mean {us.mean():.1f} max {us.max():.1f}  "
              f"add p50 {np.median(add):.1f} mean {add.mean():.1f} max {add.max():.1f}  "
              f"live {st['live_batches']} cancelled {st['live_cancelled']}  slow {slow.tolist()[:20]}", flush=True)
        for i in slow[:8]:
            print(f"   batch {i}: window {us[i]:.1f} add {add[i]:.1f}", flush=True)
    cs.close()


if __name__ == "__main__":
    main()
