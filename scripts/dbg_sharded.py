"""Debug: GPU shards vs CPU model shards, side by side, first divergence per phase."""
import random
import sys

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from foundationdb_amd.sharded import ShardedConflictSet  # noqa: E402
from gen import tiny_stream  # noqa: E402
from shard_model import ModelShard  # noqa: E402
from test_sharded import random_bounds  # noqa: E402

maxlen = int(sys.argv[1]) if len(sys.argv) > 1 else 3
nseeds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for seed in range(nseeds):
    rng = random.Random(seed * 5 + maxlen)
    G = rng.choice([2, 3, 4])
    bounds = random_bounds(rng, G, min(maxlen, 4))
    g = ShardedConflictSet(bounds, max_history=1 << 14)
    m = ShardedConflictSet(bounds, devices=[-1] * G, shard_factory=ModelShard)
    prev = None
    for i, (batch, now, nold) in enumerate(tiny_stream(seed * 13 + maxlen, n_batches=25, maxlen=maxlen)):
        vg = g.detect_packed(batch, now, nold)
        vm = m.detect_packed(batch, now, nold)
        bad = not np.array_equal(vg, vm)
        hs = [(s.history(), t.history()) for s, t in zip(g.shards, m.shards)]
        badh = [k for k, (a, b) in enumerate(hs) if a != b]
        if bad or badh or g.removal_key() != m.removal_key():
            print(f"seed {seed} batch {i} bounds {bounds} now {now} nold {nold} oldest_before {prev}")
            print("verdict gpu", vg.tolist(), "\n        mdl", vm.tolist())
            print("rk", g.removal_key(), m.removal_key())
            print("carry", [s.cs.header_version for s in g.shards], [t.v0 for t in m.shards])
            for k, (a, b) in enumerate(hs):
                print(f" shard {k} gpu {a}\n         mdl {b}")
            print("pre-batch model history per shard:", prevh)
            for t in batch.txns():
                print("  txn", t)
            sys.exit(1)
        prevh = [t.history() for t in m.shards]
        prev = m.oldest
    g.close()
print("all equal")
