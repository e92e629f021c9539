"""Load-metrics roll timing split: device roll + sync alone (nothing sampled)
vs the full call (Knobs' units), on config-2 batches resident in HBM."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from foundationdb_amd import ConflictSet
from foundationdb_amd.workload import Workload
from foundationdb_amd.load_metrics import IopsSample

cs = ConflictSet(device=0)
wl = Workload(2, txns=5000)
for units in (1 << 62, 20000, 2000):
    smp = IopsSample(units, seed=1)
    ts, n = [], 0
    for j in range(60):
        b, now, nold = wl.batch(j)
        cs.detect_packed(b, now, nold)
        t0 = time.perf_counter()
        n += smp.add_batch(cs, j * 0.01 + 1.0)
        ts.append(time.perf_counter() - t0)
        smp.poll(j * 0.01)
    ts = sorted(ts[10:])
    print(f"units={units}: median {ts[len(ts)//2]*1e6:.1f} us, min {ts[0]*1e6:.1f} us, sampled/batch {n/60:.1f}, size {smp.size()}", flush=True)
