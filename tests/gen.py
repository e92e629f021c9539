"""Random batch streams for differential tests.

Tiny alphabets with "", b"\\x00" and prefix keys make adjacent, touching,
overlapping and prefix-related ranges common; versions move forward batch to
batch while newOldest is allowed to stall or move back (non-monotone), so
tooOld, compaction windows and the removalKey wrap are all exercised.
"""
import random

from foundationdb_amd.batch import PackedBatch

ALPHA = b"ab\x00c"


def rand_key(rng, maxlen, alpha=ALPHA):
    n = rng.randint(0, maxlen)
    return bytes(rng.choice(alpha) for _ in range(n))


def rand_range(rng, maxlen, alpha=ALPHA):
    while True:
        a, b = rand_key(rng, maxlen, alpha), rand_key(rng, maxlen, alpha)
        if a != b:
            return (min(a, b), max(a, b))


def tiny_stream(seed, n_batches=30, max_txns=40, maxlen=3, max_reads=2, max_writes=2, alpha=ALPHA):
    """Yields (PackedBatch, now, new_oldest)."""
    rng = random.Random(seed)
    now = 10
    new_oldest = 0
    for _ in range(n_batches):
        now += rng.randint(1, 6)
        if rng.random() < 0.7:
            new_oldest = max(0, now - rng.randint(2, 15))
        elif rng.random() < 0.5:
            new_oldest = max(0, new_oldest - rng.randint(0, 3))
        txns = []
        for _t in range(rng.randint(0, max_txns)):
            snap = now - rng.randint(1, 20)
            reads = [rand_range(rng, maxlen, alpha) for _ in range(rng.randint(0, max_reads))]
            writes = [rand_range(rng, maxlen, alpha) for _ in range(rng.randint(0, max_writes))]
            txns.append((snap, reads, writes))
        yield PackedBatch.from_txns(txns), now, new_oldest


def mixed_stream(seed, n_batches=20, max_txns=300, keyspace=2000, wide=0.1):
    """Larger batches over a bounded integer key space with some wide ranges."""
    rng = random.Random(seed)
    now = 1000
    for _ in range(n_batches):
        now += rng.randint(50, 200)
        new_oldest = now - rng.randint(100, 800)
        txns = []

        def key(i):
            return b"k%06d" % i

        def rng_range():
            a = rng.randrange(keyspace)
            if rng.random() < wide:
                b = min(keyspace, a + rng.randint(1, keyspace // 4))
            else:
                b = a + 1
            if rng.random() < 0.5 and b == a + 1:
                return (key(a), key(a) + b"\x00")
            return (key(a), key(b))

        for _t in range(rng.randint(1, max_txns)):
            snap = now - rng.randint(1, 400)
            reads = [rng_range() for _ in range(rng.randint(0, 4))]
            writes = [rng_range() for _ in range(rng.randint(0, 3))]
            txns.append((snap, reads, writes))
        yield PackedBatch.from_txns(txns), now, new_oldest
