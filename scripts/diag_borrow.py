"""Live-ingest counts of borrowed batches in the bench's flow (GPU box):
prefill through the packed path, then Resolver windows through the native loop."""
import sys
import torch
from foundationdb_amd import ConflictSet
from foundationdb_amd.workload import Workload

torch.cuda.set_device(0)
flags = int(sys.argv[1]) if len(sys.argv) > 1 else 1
cs = ConflictSet(device=0, max_history=30_000_000, flags=flags)
wl = Workload(2, txns=5000)
wl.prefill(cs, 0, 300)
for j in range(3):
    s0 = cs.batch_stats()
    r = wl.prepare_run(300 + 40 * j, 40)
    us, add, v = r.run(cs, verdicts=False)
    s1 = cs.batch_stats()
    print(j, {k: s1[k] - s0[k] for k in ("live_batches", "live_cancelled", "live_timeouts")},
          "window us p50", sorted(us)[20], "adds", sorted(add)[20], flush=True)
