"""Protocol A/B exact sharding at the bench's scale in ONE process (every shard
on this GPU), checked against one oracle conflict set every few batches.
usage: python scripts/repro/sharded_scale.py [batches=300] [sparse=1] [G=2] [txns=10000]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from foundationdb_amd.resolvers import uniform_bounds  # noqa: E402
from foundationdb_amd.sharded import ShardedConflictSet  # noqa: E402
from foundationdb_amd.workload import Workload  # noqa: E402
from oracle import CpuSpec  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    sparse = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    T = int(sys.argv[4]) if len(sys.argv) > 4 else 10000
    sh = ShardedConflictSet(uniform_bounds(G), sparse=sparse, max_history=30_000_000)
    c = CpuSpec()
    wl = Workload(2, txns=T)
    for i in range(n):
        batch, now, nold = wl.batch(i)
        vg = sh.detect_packed(batch, now, nold)
        vc = c.detect_packed(batch, now, nold)
        assert np.array_equal(np.asarray(vg), vc), f"verdicts differ at batch {i}"
        if i % 25 == 0:
            print(f"batch {i} ok H={c.history_size()}", flush=True)
    print("done", flush=True)


if __name__ == "__main__":
    main()
