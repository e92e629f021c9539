"""Fault hunting: the in-process sharded protocol (ShardedConflictSet) on the
long-key stream of tests/test_tail_gc.py, history compared after every batch;
prints the first difference and each shard's tail-arena state.
    python scripts/repro/sharded_long_keys.py [sparse=0] [batches=60]
(FDBCS_NO_SHARD_GC=1: no tail moves in the shards)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

from foundationdb_amd.sharded import ShardedConflictSet  # noqa: E402
from oracle import CpuSpec  # noqa: E402
from test_tail_gc import PREFIX, long_key_stream  # noqa: E402


def main():
    sparse = len(sys.argv) > 1 and sys.argv[1] == "1"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    import torch
    torch.cuda.set_device(0)
    bounds = [PREFIX + b"\x80"]
    sh = ShardedConflictSet(bounds, max_history=1 << 20, sparse=sparse, tail_arena_bytes=4 << 20)
    c = CpuSpec()
    for i, (b, now, nold) in enumerate(long_key_stream(6, n)):
        v = sh.detect_packed(b, now, nold)
        vc = c.detect_packed(b, now, nold)
        st = [x.cs.batch_stats() for x in sh.shards]
        hs = [x.cs.history() for x in sh.shards]
        hc = c.history()
        desc = " | ".join(f"H={len(h)} half={s['tail_half']} used={s['tail_used']} arena={s['tail_arena_bytes']}"
                          for h, s in zip(hs, st))
        ok_v = np.array_equal(v, vc)
        hg = hs[0] + hs[1]
        ok_h = hg == hc
        print(f"batch {i}: verdicts {'ok' if ok_v else 'DIFF'} history {'ok' if ok_h else 'DIFF'} "
              f"(gpu {len(hg)} oracle {len(hc)}) rk_gpu={len(sh.removal_key())} rk_orc={len(c.removal_key())} "
              f"{desc}", flush=True)
        if not ok_h:
            for j, (a, z) in enumerate(zip(hg, hc)):
                if a != z:
                    print(f"  first diff at {j} (shard 0 holds {len(hs[0])}): gpu {a[0][-12:].hex()} v{a[1]} "
                          f"len {len(a[0])} | oracle {z[0][-12:].hex()} v{z[1]} len {len(z[0])}")
                    print("  gpu around:", [(k[-6:].hex(), x) for k, x in hg[max(0, j - 2):j + 3]])
                    print("  orc around:", [(k[-6:].hex(), x) for k, x in hc[max(0, j - 2):j + 3]])
                    break
            break
        if not ok_v:
            print("  verdict diffs:", np.nonzero(v != vc)[0][:10])
            break


if __name__ == "__main__":
    main()
