"""The bench's N > 1 exact path (DistShardedConflictSet over torch.distributed,
one HIP shard per rank) checked against one oracle conflict set: verdicts
every batch (rank 0), concatenated histories at the end.
usage: python tests/dist_hip_verify.py [world=2] [batches=120] [txns=10000] [sparse=1]
(tests/test_sharded.py::test_dist_sharded_hip_engines runs it; every rank uses
GPU 0 -- the test box has one -- and gloo carries the exchanges)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(rank, world, port, n, T, sparse, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import numpy as np
    import torch
    import torch.distributed as dist
    from foundationdb_amd.batch import DeviceBatch
    from foundationdb_amd.resolvers import KeyRangeResolvers, uniform_bounds
    from foundationdb_amd.sharded import DistShardedConflictSet
    from foundationdb_amd.workload import Workload

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bounds = uniform_bounds(world)
    eng = DistShardedConflictSet(bounds, rank, world, 0, max_history=30_000_000, sparse=sparse)
    kr = KeyRangeResolvers(bounds) if sparse else None
    wl = Workload(2, txns=T)
    c = None
    if rank == 0:
        sys.path.insert(0, ROOT)
        from oracle import CpuSpec
        c = CpuSpec()
    verd = torch.empty(T, dtype=torch.uint8, device=dev)
    bad = None
    for i in range(n):
        batch, now, nold = wl.batch(i)
        sub = kr.split(batch, rank, keep_all=True)[0] if sparse else batch
        db = DeviceBatch(sub.view(), dev)
        eng.detect_device(db.view, now, nold, verd)
        torch.cuda.synchronize()
        if rank == 0:
            vc = c.detect_packed(batch, now, nold)
            vg = verd.cpu().numpy()[:batch.T]
            if bad is None and not np.array_equal(vg, vc):
                bad = (i, int((vg != vc).sum()))
                print(f"rank0: verdicts differ at batch {i}: {bad[1]} txns", flush=True)
            if i % 20 == 0:
                print(f"batch {i} H_oracle={c.history_size()} ok={bad is None}", flush=True)
    h = eng.shard.cs.history_size()
    hs = [None] * world
    dist.all_gather_object(hs, h)
    if rank == 0:
        print(f"history sizes {hs} sum {sum(hs)} oracle {c.history_size()}", flush=True)
        q.put((bad, sum(hs), c.history_size()))
    dist.destroy_process_group()


def main():
    import multiprocessing as mp
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 120
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
    sparse = bool(int(sys.argv[4])) if len(sys.argv) > 4 else True
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 300
    ps = [ctx.Process(target=rank_main, args=(r, world, port, n, T, sparse, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join()
    res = q.get() if not q.empty() else None
    print("result", res, "exit codes", [p.exitcode for p in ps], flush=True)
    ok = res is not None and res[0] is None and res[1] == res[2] and all(p.exitcode == 0 for p in ps)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
