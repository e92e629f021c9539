# The smoke() sequence with a print after every call (heap corruption hunt).
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch
torch.cuda.set_device(0)
from foundationdb_amd import ConflictSet
from foundationdb_amd.workload import Workload
from oracle import CpuSpec
skip = set(sys.argv[1:])
g = ConflictSet(device=0)
c = CpuSpec()
wl = Workload(2, txns=500)
for i in range(5):
    batch, now, nold = wl.batch(i)
    vg = g.detect_packed(batch, now, nold)
    vc = c.detect_packed(batch, now, nold)
print("detected", flush=True)
for name, fn in [("ghist", lambda: g.history()), ("chist", lambda: c.history()), ("grk", lambda: g.removal_key()),
                 ("crk", lambda: c.removal_key()), ("gsize", lambda: g.history_size()), ("close", lambda: g.close())]:
    if name in skip:
        continue
    fn()
    print(name, flush=True)
print("exiting", flush=True)
