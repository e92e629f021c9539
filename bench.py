"""Resolver conflict-detection benchmark (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2]

A step = one ConflictBatch (addTransaction x T + detectConflicts) over one
synthetic batch already staged in HBM; detectConflicts is synchronous, as the
Resolver needs the verdicts before replying (Resolver.actor.cpp:139-166).
Workload (BASELINE.json configs[1]): config 2 = 5,000 txns per
batch, 5 reads + 2 point writes per txn, uniform 16-byte keys, 5M-version MVCC
window; W warmup batches grow the history to steady state (~19 M boundaries
after ~2,500 batches), then K measured batches.

Prints ONE JSON line (rank 0).  `value` = resolved txns/s over the timed
region (max over ranks), `p99_batch_ms` = p99 per-batch detectConflicts
latency.  `roofline` is for the dominant kernel;
`cpu_baseline` times the CPU oracle (oracle/cpu_spec.cpp, 1 core) on the
same measured batches starting from the GPU's own steady-state history, and
cross-checks its verdicts against the GPU's.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=2500)
    p.add_argument("--config", type=int, default=2)
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--stage-timing", type=int, default=1)
    return p.parse_args()


def stage_batches(wl, first, k, torch, dev):
    """Generate batches [first, first+k) and copy them into device memory."""
    from foundationdb_amd._abi import BatchView
    staged = []
    for i in range(first, first + k):
        v, now, nold = wl.view(i)
        T, R, W = v.txn_count, v.read_count, v.write_count
        slots = 2 * (R + W)

        def to_dev(ptr, ctype, n, dtype):
            a = np.ctypeslib.as_array((ctype * max(n, 1)).from_address(ptr))[:n].astype(dtype, copy=True)
            return torch.from_numpy(a).to(dev)

        bufs = [to_dev(v.snapshot, C.c_int64, T, np.int64), to_dev(v.read_off, C.c_int32, T + 1, np.int32),
                to_dev(v.write_off, C.c_int32, T + 1, np.int32), to_dev(v.key_off, C.c_uint64, slots, np.int64),
                to_dev(v.key_len, C.c_uint32, slots, np.int32),
                to_dev(v.key_bytes, C.c_uint8, int(v.key_bytes_len), np.uint8)]
        dv = BatchView()
        dv.txn_count, dv.read_count, dv.write_count = T, R, W
        dv.snapshot, dv.read_off, dv.write_off = bufs[0].data_ptr(), bufs[1].data_ptr(), bufs[2].data_ptr()
        dv.key_off, dv.key_len, dv.key_bytes = bufs[3].data_ptr(), bufs[4].data_ptr(), bufs[5].data_ptr()
        dv.key_bytes_len = int(v.key_bytes_len)
        staged.append((dv, now, nold, bufs, int(v.key_bytes_len)))
    return staged


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from foundationdb_amd import ConflictSet
    from foundationdb_amd.workload import Workload

    cfg = args.config
    wl = Workload(cfg)
    cs = ConflictSet(device=local, max_history=30_000_000)

    # ---- warmup: grow the history to steady state (untimed) ----------------
    t_w = time.time()
    verdict_host = None
    for i in range(args.warmup):
        v, now, nold = wl.view(i)
        verdict_host = cs.detect_view(v, now, nold, verdict_host)
        if rank == 0 and (i + 1) % 500 == 0:
            print(f"# warmup {i + 1}/{args.warmup} H={cs.history_size()} {time.time() - t_w:.1f}s",
                  file=sys.stderr, flush=True)
    H_pre = cs.history_size()

    # CPU baseline needs the GPU's steady state: snapshot it before timing
    snap = None
    if not args.no_cpu and rank == 0 and world == 1:
        snap = cs.dump_arrays() + (cs.header_version, cs.oldest_version, cs.removal_key())

    # ---- stage K measured batches in HBM --------------------------------------
    staged = stage_batches(wl, args.warmup, args.steps, torch, dev)
    T = staged[0][0].txn_count
    verdicts = torch.zeros((args.steps, max(T, 1)), dtype=torch.uint8, device=dev)
    cs.enable_stage_timing(bool(args.stage_timing))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    # ---- timed region -----------------------------------------------------------
    lat = []
    stages = []
    t0 = time.perf_counter()
    for k, (dv, now, nold, _bufs, _nb) in enumerate(staged):
        ts = time.perf_counter()
        cs.detect_device(dv, now, nold, verdicts[k].data_ptr(), sync=True)
        lat.append(time.perf_counter() - ts)
        if args.stage_timing:
            stages.append(cs.stage_times())
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    H_post = cs.history_size()
    total_txns = T * args.steps * world
    value = total_txns / elapsed
    lat_ms = np.array(lat) * 1e3

    # ---- roofline (dominant stage) ----------------------------------------------
    roofline = None
    if stages:
        st = np.array(stages)  # [K, 7] us: sort/encode, read, intra, combine, merge, compact, total
        names = ["encode", "read_check", "intra_batch", "combine", "merge", "compaction"]
        mean = st.mean(axis=0)
        dom = int(np.argmax(mean[:6]))
        key_bytes = float(np.mean([s[4] for s in staged]))
        # SURVEY.md §8d algorithmic bytes per batch: inputs + verdicts + 28 B x (H_pre + H_post)
        algo_batch = key_bytes + 9.0 * T + 28.0 * (H_pre + H_post) / 1.0
        roofline = {
            "bound": "hbm",
            "kernel": names[dom],
            "stage_us": {n: round(float(mean[i]), 2) for i, n in enumerate(names)},
            "batch_us": round(float(mean[6]), 2),
            "achieved": round(algo_batch / (mean[6] * 1e-6) / 1e9, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "traffic": None,
        }
        roofline["frac"] = round(roofline["achieved"] / HBM_PEAK_GBS, 4)

    # ---- CPU baseline (oracle, 1 core) on the same batches, same start state -----
    cpu = None
    if snap is not None:
        from oracle import CpuSpec
        from foundationdb_amd.workload import Workload as W2
        vers, lens, offs, kb, v0, oldest, rk = snap
        c = CpuSpec()
        c.load_history_arrays(len(vers), vers, lens, offs, kb, v0=v0, oldest=oldest, removal_key=rk)
        wl2 = W2(cfg)
        n, mism, tc = 0, 0, 0.0
        gv = verdicts.cpu().numpy()
        while n < args.steps and tc < args.cpu_seconds:
            b, now, nold = wl2.batch(args.warmup + n)
            ts = time.perf_counter()
            vc = c.detect_packed(b, now, nold)
            tc += time.perf_counter() - ts
            mism += int((vc != gv[n][:T]).sum())
            n += 1
        cpu = {"value": round(n * T / tc, 1), "unit": "txn/s", "cores": 1, "kind": "port",
               "sample": f"config {cfg}: batches {args.warmup}..{args.warmup + n - 1} ({n} x {T} txns) from the "
                         f"GPU's steady-state history (H={H_pre}); verdict mismatches vs GPU: {mism}"}

    if rank == 0:
        out = {
            "metric": "resolved txns/sec (whole node) at 5k-txn batches; p99 detectConflicts latency",
            "value": round(value, 1),
            "unit": "txn/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "p99_batch_ms": round(float(np.percentile(lat_ms, 99)), 4),
            "p50_batch_ms": round(float(np.percentile(lat_ms, 50)), 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (deterministic generator, SURVEY.md §8d)",
            "config": {"workload": f"config{cfg}: {T}-txn batches, 5R+2W, uniform 16-byte keys, 5M-version window",
                       "txns_per_batch": T, "history_pre": H_pre, "history_post": H_post,
                       "parallelism": f"keyrange{world}" if world > 1 else "single"},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
