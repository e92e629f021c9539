"""Load-metrics roll timing split: device roll + sync alone (nothing sampled)
vs the full call (Knobs' units), on config-2 batches resident in HBM."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foundationdb_amd import ConflictSet
from foundationdb_amd.workload import Workload
from foundationdb_amd.load_metrics import IopsSample

cs = ConflictSet(device=0)
wl = Workload(2, txns=int(sys.argv[1]) if len(sys.argv) > 1 else 5000)
for units in ((1 << 62, 20000) if len(sys.argv) > 1 else (1 << 62, 20000, 2000)):
    smp = IopsSample(units, seed=1)
    ts, n = [], 0
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    for j in range(nb):
        b, now, nold = wl.batch(j)
        cs.detect_packed(b, now, nold)
        t0 = time.perf_counter()
        n += smp.add_batch(cs, j * 0.01 + 1.0)
        ts.append(time.perf_counter() - t0)
        smp.poll(j * 0.01)
    ts = sorted(ts[len(ts) // 6:])
    print(f"units={units}: median {ts[len(ts)//2]*1e6:.1f} us, min {ts[0]*1e6:.1f} us, sampled/batch {n/nb:.1f}, size {smp.size()}", flush=True)
