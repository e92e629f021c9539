# Locate the heap corruption seen at the end of __graft_entry__.smoke().
import sys, os, faulthandler
faulthandler.enable()
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch
step = sys.argv[1] if len(sys.argv) > 1 else "all"
print("cuda", torch.cuda.is_available(), flush=True)
torch.cuda.set_device(0)
from foundationdb_amd import ConflictSet
from foundationdb_amd.workload import Workload
print("imported", flush=True)
if step in ("build", "oracle"):
    import __graft_entry__ as GE
    if step == "build":
        GE.build()
        print("built", flush=True)
c = None
if step == "oracle":
    from oracle import CpuSpec
    c = CpuSpec()
g = ConflictSet(device=0)
print("created", flush=True)
wl = Workload(2, txns=500)
for i in range(5):
    batch, now, nold = wl.batch(i)
    vg = g.detect_packed(batch, now, nold)
    if c is not None:
        vc = c.detect_packed(batch, now, nold)
print("detected", flush=True)
if step in ("all", "close", "oracle", "build"):
    g.close()
    print("closed", flush=True)
if step in ("all",):
    del wl
    print("wl deleted", flush=True)
print("exiting", flush=True)
