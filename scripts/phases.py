"""Print intra-kernel phase timings (profiling build, FDBCS_PHASES=1).

usage: bash scripts/build_variants.sh phases:-DFDBCS_PHASES
       FDBCS_LIB_PATH=scripts/micro/var/libfdbcs_phases.so python scripts/phases.py [warmup] [batches] [config]
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foundationdb_amd import ConflictSet  # noqa: E402
from foundationdb_amd.workload import Workload  # noqa: E402


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    cs = ConflictSet(device=0, max_history=30_000_000)
    wl = Workload(int(sys.argv[3]) if len(sys.argv) > 3 else 2)
    out = None
    for i in range(warm):
        v, now, nold = wl.view(i)
        out = cs.detect_view(v, now, nold, out)
    acc, stats = [], []
    buf = (C.c_int64 * 32)()
    for i in range(warm, warm + nb):
        v, now, nold = wl.view(i)
        out = cs.detect_view(v, now, nold, out)
        n = cs._lib.fdbcs_debug_phases(cs.handle, buf, 32)
        if n <= 0:
            print("not a FDBCS_PHASES build")
            return
        acc.append(np.array(buf[:n], dtype=np.int64))
        st = cs.batch_stats()
        stats.append((st.get("dependents", 0), st.get("decision_rounds", 0)))
    a = np.array(acc)
    base = a[:, 0:1]
    d = (a - base) * 0.01  # 100 MHz ticks -> us
    m = d.mean(axis=0)
    print(f"H={cs.history_size()}  phase offsets (us from phase 0), mean over {nb} batches:")
    for i in range(min(16, a.shape[1])):
        if a[:, i].any():
            print(f"  ph[{i:2d}] {m[i]:9.2f}  (+{m[i] - (m[i - 1] if i else 0):8.2f})")
    sd = np.array(stats)
    print(f"  decision: candidate reads mean {sd[:, 0].mean():.1f} (batches with any: {(sd[:, 0] > 0).sum()}), "
          f"rounds mean {sd[:, 1].mean():.2f}")
    if a.shape[1] > 16:  # cumulative per-wave cycle accumulators: per-batch deltas
        dd = np.diff(a[:, 16:], axis=0).mean(axis=0)
        print("  accumulators per batch:", " ".join(f"[{16 + i}]={v:.0f}" for i, v in enumerate(dd) if v))


if __name__ == "__main__":
    main()
