"""Diagnosis run for round 3's one-off sharded history drop.

test_gpu_shards_tiny_streams[11-False] once lost the committed begin at ""
in shard 0's first batch (seed 0: bounds [cbac, ccbb], now=14).  This runs
that first batch on N freshly created shard sets (fresh device memory every
time, as the test family does) and, on the first mismatch, prints every
shard's batch statistics (combined ranges, pages merged, directory entries,
history) so the failing stage can be named.  One bounded run:

    python scripts/repro/sharded_first_batch.py [N]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from foundationdb_amd.sharded import ShardedConflictSet  # noqa: E402
from oracle import CpuSpec  # noqa: E402
from test_sharded import first_batch_cases  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    cases = list(first_batch_cases())
    bad = 0
    for it in range(n):
        for ci, (bounds, batch, now, nold) in enumerate(cases):
            for sparse in (False, True):
                sh = ShardedConflictSet(bounds, max_history=1 << 14, sparse=sparse)
                c = CpuSpec()
                try:
                    vs = sh.detect_packed(batch, now, nold)
                    vc = c.detect_packed(batch, now, nold)
                    hs, hc = sh.history(), c.history()
                    if (vs != vc).any() or hs != hc:
                        bad += 1
                        print(f"MISMATCH it={it} case={ci} sparse={sparse}: verdicts_equal={(vs == vc).all()}")
                        print(f"  gpu    {hs}")
                        print(f"  oracle {hc}")
                        for g, s in enumerate(sh.shards):
                            print(f"  shard {g} [{s.lo!r}, {s.hi!r}): {s.cs.batch_stats()} H={s.cs.history_size()}")
                        sys.stdout.flush()
                        return 1
                finally:
                    sh.close()
                    c.close()
        if (it + 1) % 20 == 0:
            print(f"# {it + 1}/{n} rounds clean", flush=True)
    print(f"clean: {n} rounds x {len(cases)} cases x 2 protocols")
    return 0


if __name__ == "__main__":
    sys.exit(main())
