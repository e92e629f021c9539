"""Resolver conflict-detection benchmark (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2]
    torchrun --nproc-per-node N bench.py --gpus N ...      (N > 1)

A step = one ConflictBatch (addTransaction x T + detectConflicts) over one
synthetic batch already staged in HBM; detectConflicts is synchronous, as the
Resolver needs the verdicts before replying (Resolver.actor.cpp:139-166).

N = 1: BASELINE.json configs[1] = SURVEY.md §8d config 2: 5,000-txn batches,
5 reads (80 % point, 20 % short) + 2 point writes per txn, uniform 16-byte
keys, 5M-version MVCC window; W warmup batches grow the history to steady
state (~19 M boundaries after ~2,500 batches), then K measured batches.

N > 1, --mode exact (default; the north star's layout, SURVEY.md §8e
protocol A): ONE resolver over N GPUs.  GPU g holds the history of the g-th
equal slice of the key space; every GPU receives the whole global batch of
5,000 x N transactions, checks the reads clipped to its keys, an RCCL MAX
all-reduce combines the per-transaction conflict flags, every GPU replays the
identical ordered decision and merges its shard's part of the committed
writes, and two tiny all-gathers drive the global compaction window.  The
verdicts and the concatenated history equal a single conflict set's exactly.
Per-GPU history and merge work stay ~fixed (weak scaling); the batch-wide
stages (ingest, sort, decision) see the whole N x 5,000 batch on every GPU.

N > 1, --mode resolvers: FoundationDB's multi-resolver scale-out (SURVEY.md
§3.4): GPU g is an independent resolver for the g-th key slice; the global
batch is split by the proxy rule (fdbcs_split_batch,
MasterProxyServer.actor.cpp:267-307), every GPU resolves its sub-batch, and
the proxy's min-combine (:558-569) is a scatter + RCCL MIN all-reduce of the
verdict bytes inside the timed step (conservative, as FDB's own).

Prints ONE JSON line (rank 0).  `value` = resolved txns/s (whole node, max
time over ranks), `p99_batch_ms` = p99 per-batch latency.  `roofline`: the
pipeline of one detectConflicts (all its kernels, bracketed by HIP events on
the conflict set's stream) against the HBM peak, with SURVEY.md §8d's
algorithmic bytes per batch; `dominant_stage` gives the longest stage with its
own byte model.  `cpu_baseline` times the CPU oracle
(oracle/cpu_spec.cpp, 1 core) on the same measured batches starting from the
GPU's own steady-state history, and cross-checks its verdicts.
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
STAGES = ["encode", "sort", "read_check_edges", "decide_combine", "merge", "compaction"]
E_HIST = 28.0  # SURVEY.md §8d bytes per boundary (16-B prefix + 8-B version + 4-B meta)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="measured batches (default 200; config 5: 10)")
    p.add_argument("--warmup", type=int, default=None,
                   help="untimed batches before them (default 2500; config 5: 2, after the 10^8-boundary preload)")
    p.add_argument("--config", type=int, default=2)
    p.add_argument("--txns", type=int, default=None, help="transactions per batch per GPU (default 5000; config 5: 10^6)")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--stage-batches", type=int, default=None,
                   help="extra instrumented batches after the timed region (default 50; config 5: 3)")
    p.add_argument("--mode", choices=["exact", "resolvers"], default="exact",
                   help="N > 1: one exact resolver sharded by key range, or N independent key-range resolvers")
    p.add_argument("--pcie-batches", type=int, default=None,
                   help="host batches timed through the PCIe-inclusive paths after the measurement (default 50; "
                        "config 5: 2)")
    p.add_argument("--lm-batches", type=int, default=None,
                   help="batches whose load-metrics roll (iopsSample, Resolver.actor.cpp:146-151) is timed after "
                        "the measurement (default 50; config 5: 2)")
    p.add_argument("--protocol", choices=["a", "b"], default="b",
                   help="exact mode: A = every GPU receives the whole batch; B = each GPU receives only the ranges "
                        "intersecting its keys and the overlap edges are all-gathered (SURVEY.md §8e)")
    a = p.parse_args()
    big = a.config == 5  # 1 M-txn batches over a preloaded 10^8-boundary history
    for name, small, large in [("steps", 200, 10), ("warmup", 2500, 2), ("txns", 5000, 1_000_000),
                               ("stage_batches", 50, 3), ("pcie_batches", 50, 2),
                               ("lm_batches", 50, 2)]:
        if getattr(a, name) is None:
            setattr(a, name, large if big else small)
    return a


PRELOAD_BATCHES = 50  # config 5: 50 blind-write batches of 10^6 point writes


def max_history(cfg):
    return 130_000_000 if cfg == 5 else 30_000_000


def to_device(v, torch, dev):
    """Copy a host fdbcs_batch_view into device tensors; returns (device view, keepalive)."""
    from foundationdb_amd._abi import BatchView
    T, R, W = v.txn_count, v.read_count, v.write_count
    slots = 2 * (R + W)

    def arr(ptr, ctype, n, dtype):
        if n == 0:
            return torch.zeros(1, dtype=torch.uint8, device=dev)
        a = np.ctypeslib.as_array((ctype * n).from_address(ptr)).astype(dtype, copy=True)
        return torch.from_numpy(a).to(dev)

    bufs = [arr(v.snapshot, C.c_int64, T, np.int64), arr(v.read_off, C.c_int32, T + 1, np.int32),
            arr(v.write_off, C.c_int32, T + 1, np.int32), arr(v.key_off, C.c_uint64, slots, np.int64),
            arr(v.key_len, C.c_uint32, slots, np.int32), arr(v.key_bytes, C.c_uint8, int(v.key_bytes_len), np.uint8)]
    dv = BatchView()
    dv.txn_count, dv.read_count, dv.write_count = T, R, W
    dv.snapshot, dv.read_off, dv.write_off = bufs[0].data_ptr(), bufs[1].data_ptr(), bufs[2].data_ptr()
    dv.key_off, dv.key_len, dv.key_bytes = bufs[3].data_ptr(), bufs[4].data_ptr(), bufs[5].data_ptr()
    dv.key_bytes_len = int(v.key_bytes_len)
    return dv, bufs


class Source:
    """Batches for this rank: the whole batch (N = 1) or this resolver's share."""

    def __init__(self, cfg, txns, world, rank, split, keep_all=False):
        from foundationdb_amd.workload import Workload
        self.world, self.rank = world, rank
        self.wl = Workload(cfg, txns=txns * world)
        self.kr = None
        self.keep_all = keep_all  # protocol B: every transaction, only this rank's ranges
        if split and world > 1:
            from foundationdb_amd.resolvers import KeyRangeResolvers, uniform_bounds
            self.kr = KeyRangeResolvers(uniform_bounds(world))

    def host(self, i):
        """(host view, now, new_oldest, T_global, txn_index or None, keepalive)."""
        if self.kr is None:
            v, now, nold = self.wl.view(i)
            return v, now, nold, v.txn_count, None, None
        batch, now, nold = self.wl.batch(i)
        sub, idx = self.kr.split(batch, self.rank, keep_all=self.keep_all)
        return sub.view(), now, nold, batch.T, (None if self.keep_all else idx), (sub, batch)


CONFIG_SHAPE = {
    1: "skiplisttest keys (12 x '.' + BE32), 1R+1W",
    2: "5R+2W, uniform 16-byte keys",
    3: "5R+2W, Zipf(0.99) hot 16-byte keys over 10^6 ranks (long intra-batch chains)",
    4: "4 point reads + 1 wide read (10^3-10^5 boundaries) + 2W, 68-100-byte keys (tail compares)",
    5: "5R+2W, uniform 16-byte keys, history preloaded to 10^8 boundaries (50 blind-write batches of 10^6)",
}


def pipeline_bytes(key_bytes, T, h_pre, h_post, cfg=2):
    """SURVEY.md §8d algorithmic bytes per batch: inputs + 8 T snapshots + T
    verdicts + E (H_pre + H_post) (history read once, written once); E = 28 B
    for keys <= 17 B, 32 B (8-B meta with a tail offset) for config 4."""
    e = 32.0 if cfg == 4 else E_HIST
    return key_bytes + 9.0 * T + e * (h_pre + h_post)


def stage_bytes(name, st, key_bytes):
    """Bytes each stage must move in this design."""
    T, R, W = st["txns"], st["reads"], st["writes"]
    fill = st["history"] / max(1, st["dir_entries"])
    if name == "merge":  # rewrite the touched pages + the directory
        return 2 * st["pages_merged"] * fill * 36.0 + 2 * st["dir_entries"] * 52.0 + st["combined"] * 64.0
    if name == "compaction":
        return st["window_pages"] * fill * 36.0 + st["window_survivors"] * 36.0 + 2 * st["dir_entries"] * 52.0
    if name == "read_check_edges":  # history search per read + the sorted endpoints the edges search
        return R * (2 * 24.0 + 4 + 8 + 2 * 36.0) + T + (R + W) * 48.0
    if name == "sort":
        return (R + 2 * W) * (24.0 + 4 * 32.0)
    if name == "decide_combine":
        return T * 8.0 + 2 * W * (4.0 + 8.0)
    return key_bytes + 2 * (R + W) * 24.0  # encode


def time_resolvers(args, world, rank, dev, torch, dist):
    """N > 1 supplement: the same global batches through FDB's key-range
    resolvers (--mode resolvers), for the line's `alt_modes` field."""
    from foundationdb_amd import ConflictSet
    from foundationdb_amd.resolvers import scatter_verdicts

    src = Source(args.config, args.txns, world, rank, split=True)
    cs = ConflictSet(device=dev.index, max_history=max_history(args.config))
    out = None
    for i in range(args.warmup):
        v, now, nold, _T, _idx, _keep = src.host(i)
        out = cs.detect_view(v, now, nold, out)
    staged = []
    for i in range(args.warmup, args.warmup + args.steps):
        v, now, nold, Tg, idx, keep = src.host(i)
        dv, bufs = to_device(v, torch, dev)
        staged.append((dv, now, nold, Tg, torch.from_numpy(idx).to(dev), bufs))
        del keep
    Tg = staged[0][3]
    sub = torch.zeros((args.steps, max(1, max(x[0].txn_count for x in staged))), dtype=torch.uint8, device=dev)
    full = torch.full((args.steps, max(Tg, 1)), 2, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    dist.barrier()
    lat = []
    t0 = time.perf_counter()
    for k, (dv, now, nold, _Tg, didx, _b) in enumerate(staged):
        ts = time.perf_counter()
        cs.detect_device(dv, now, nold, sub[k].data_ptr(), sync=True)
        scatter_verdicts(None, sub[k].data_ptr(), didx.data_ptr(), dv.txn_count, full[k].data_ptr())
        dist.all_reduce(full[k], op=dist.ReduceOp.MIN)
        torch.cuda.current_stream().synchronize()
        lat.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    cs.close()
    return {"mode": "resolvers", "value": round(Tg * args.steps / elapsed, 1), "unit": "txn/s",
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "p99_batch_ms": round(float(np.percentile(np.array(lat) * 1e3, 99)), 4),
            "semantics": f"{world} independent key-range resolvers (FDB's own scale-out; conservative, not "
                         f"bit-exact to one resolver)"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # RCCL over xGMI; FDBCS_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs
        backend = os.environ.get("FDBCS_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from foundationdb_amd import ConflictSet
    from foundationdb_amd.batch import DeviceBatch
    from foundationdb_amd.resolvers import scatter_verdicts, uniform_bounds

    cfg = args.config
    mode = args.mode if world > 1 else "single"
    sparse = mode == "exact" and args.protocol == "b"
    src = Source(cfg, args.txns, world, rank, split=(mode == "resolvers" or sparse), keep_all=sparse)
    eng = None
    if mode == "exact":
        from foundationdb_amd.sharded import DistShardedConflictSet
        eng = DistShardedConflictSet(uniform_bounds(world), rank, world, local, max_history=max_history(cfg),
                                     sparse=sparse)
        cs = eng.shard.cs
    else:
        cs = ConflictSet(device=local, max_history=max_history(cfg))

    def global_h():
        """History size of the whole resolver (the sum over shards in exact mode)."""
        if mode != "exact":
            return cs.history_size()
        return sum(x[0] for x in eng._allgather([cs.history_size()]))

    # ---- warmup: grow the history to steady state (untimed) ----------------
    t_w = time.time()
    verdict_host = None
    wverd = None
    pre = None
    if cfg == 5:  # preload: blind-write batches (config 50 of the generator), no compaction
        pre = Source(50, args.txns, world, rank, split=(mode == "resolvers" or sparse), keep_all=sparse)
    n_pre = PRELOAD_BATCHES if pre is not None else 0
    for j in range(n_pre + args.warmup):
        i = j - n_pre
        v, now, nold, _T, _idx, _keep = (pre.host(j) if i < 0 else src.host(i))
        if mode == "exact":
            db = DeviceBatch(v, dev)
            if wverd is None or wverd.numel() < max(1, v.txn_count):
                wverd = torch.empty(max(1, v.txn_count), dtype=torch.uint8, device=dev)
            eng.detect_device(db.view, now, nold, wverd)
        else:
            verdict_host = cs.detect_view(v, now, nold, verdict_host)
        if rank == 0 and ((j + 1) % 500 == 0 or pre is not None):
            print(f"# warmup {j + 1}/{n_pre + args.warmup} H={cs.history_size()} {time.time() - t_w:.1f}s",
                  file=sys.stderr, flush=True)
    H_pre = global_h()
    H_pre_local = cs.history_size()

    # CPU baseline needs the GPU's steady state: snapshot it before timing
    snap = None
    if not args.no_cpu and rank == 0 and world == 1:
        snap = cs.dump_arrays() + (cs.header_version, cs.oldest_version, cs.removal_key())

    # ---- stage the K measured batches (+ instrumented ones) in HBM -------------
    n_stage = args.steps + (args.stage_batches if mode != "exact" else 0)
    staged = []
    for i in range(args.warmup, args.warmup + n_stage):
        v, now, nold, Tg, idx, keep = src.host(i)
        dv, bufs = to_device(v, torch, dev)
        didx = torch.from_numpy(idx).to(dev) if idx is not None else None
        staged.append((dv, now, nold, Tg, didx, bufs, int(v.key_bytes_len)))
        del keep
    Tg = staged[0][3]
    Tmax = max(max(s[0].txn_count for s in staged), 1)
    sub_verdicts = torch.zeros((args.steps, Tmax), dtype=torch.uint8, device=dev)
    global_verdicts = torch.full((args.steps, max(Tg, 1)), 2, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    if mode == "exact" and os.environ.get("FDBCS_PHASES_HOST"):
        eng.enable_phase_timing(True)
    # ---- timed region: K steps -------------------------------------------------
    if os.environ.get("FDBCS_VERBOSE"):
        print(f"# rank {rank}: timed region starts", file=sys.stderr, flush=True)
    lat = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        dv, now, nold, _Tg, didx, _b, _nb = staged[k]
        ts = time.perf_counter()
        if mode == "exact":  # one resolver over N GPUs: check, MAX all-reduce, decide + merge, compaction
            eng.detect_device(dv, now, nold, sub_verdicts[k])
        else:
            cs.detect_device(dv, now, nold, sub_verdicts[k].data_ptr(), sync=True)
        if mode == "resolvers":  # proxy combine: scatter this resolver's verdicts, MIN over resolvers
            scatter_verdicts(None, sub_verdicts[k].data_ptr(), didx.data_ptr(), dv.txn_count,
                             global_verdicts[k].data_ptr())
            dist.all_reduce(global_verdicts[k], op=dist.ReduceOp.MIN)
            torch.cuda.current_stream().synchronize()
        lat.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    alt = None
    if mode == "exact" and os.environ.get("FDBCS_BENCH_ALT", "1") != "0":
        alt = {"resolvers": time_resolvers(args, world, rank, dev, torch, dist)}
    if eng is not None and eng.phase_s:
        print(f"# rank {rank} phase us/batch: " +
              json.dumps({k: round(v / args.steps * 1e6, 1) for k, v in eng.phase_s.items()}), file=sys.stderr,
              flush=True)
    H_post = global_h()
    H_post_local = cs.history_size()
    total_txns = Tg * args.steps
    value = total_txns / elapsed
    lat_ms = np.array(lat) * 1e3

    # ---- instrumented pass: per-stage HIP-event times on the engine's stream ---
    roofline = None
    if mode == "exact":  # per-GPU algorithmic bytes (its shard's history) over the per-batch wall time
        nbytes = float(np.mean([x[6] for x in staged[:args.steps]]))
        algo = pipeline_bytes(nbytes, Tg, H_pre_local, H_post_local, cfg)
        batch_us = elapsed / args.steps * 1e6
        achieved = algo / (batch_us * 1e-6) / 1e9
        roofline = {
            "bound": "hbm",
            "kernel": "detectConflicts pipeline per GPU (whole batch + its shard's history; SURVEY §8d bytes), "
                      "wall time per batch including the RCCL exchanges",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "algo_bytes_per_batch": round(algo),
            "batch_us": round(batch_us, 2),
            "shard_history_pre": H_pre_local,
        }
    if args.stage_batches > 0 and mode != "exact":
        cs.enable_stage_timing(True)
        st_us, stats, hp = [], [], []
        scratch = torch.zeros(Tmax, dtype=torch.uint8, device=dev)
        for k in range(args.steps, n_stage):
            dv, now, nold, _Tg, _didx, _b, nbytes = staged[k]
            h0 = cs.history_size()
            cs.detect_device(dv, now, nold, scratch.data_ptr(), sync=True)
            st_us.append(cs.stage_times())
            stats.append(cs.batch_stats())
            hp.append((h0, cs.history_size(), nbytes, dv.txn_count))
        cs.enable_stage_timing(False)
        mean = np.array(st_us).mean(axis=0)  # [6 stages..., whole batch] us
        batch_us = float(mean[6])
        algo = float(np.mean([pipeline_bytes(nb, T, a, b, cfg) for a, b, nb, T in hp]))
        dom = int(np.argmax(mean[:6]))
        dom_bytes = float(np.mean([stage_bytes(STAGES[dom], s, nb) for s, (_a, _b, nb, _T) in zip(stats, hp)]))
        achieved = algo / (batch_us * 1e-6) / 1e9
        roofline = {
            "bound": "hbm",
            "kernel": "detectConflicts pipeline (one batch, all stages; SURVEY §8d bytes)",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "algo_bytes_per_batch": round(algo),
            "batch_us": round(batch_us, 2),
            "stage_us": {n: round(float(mean[i]), 2) for i, n in enumerate(STAGES)},
            "dominant_stage": {
                "name": STAGES[dom],
                "us": round(float(mean[dom]), 2),
                "bytes": round(dom_bytes),
                "achieved": round(dom_bytes / (mean[dom] * 1e-6) / 1e9, 1),
                "frac": round(dom_bytes / (mean[dom] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            },
            "measured_over": f"{args.stage_batches} batches after the timed region (HIP events per stage)",
            "sort_rebucketed_batches": int(sum(x.get("sort_rebucketed", 0) for x in stats)),
            "sort_max_bucket": int(max(x.get("sort_max_bucket", 0) for x in stats)),
        }
        prof = os.path.join(ROOT, "profiles", f"pmc_traffic_config{cfg}.json")
        if os.path.exists(prof):  # per-batch HBM bytes from separate rocprofv3 --pmc passes
            with open(prof) as f:
                pm = json.load(f)
            roofline["traffic"] = pm.get("bytes_per_batch")
            roofline["traffic_source"] = pm.get("source")

    # ---- PCIe-inclusive rate (not `value`): host SoA batches through the C ABI ----
    pcie = None
    if mode == "single" and args.pcie_batches > 0:
        n = args.pcie_batches
        first = args.warmup + n_stage
        host = [src.wl.batch(first + j) for j in range(2 * n + 2)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b, now, nold in host[:n]:  # synchronous: pack, H2D, pipeline, verdict D2H, then the next
            cs.detect_packed(b, now, nold)
        t_serial = time.perf_counter() - t0
        cs.submit_packed(*host[n])  # (untimed: sizes both of the pipelined path's staging slots)
        cs.submit_packed(*host[n + 1])
        cs.wait()
        cs.wait()
        t0 = time.perf_counter()
        for j, (b, now, nold) in enumerate(host[n + 2:]):  # two in flight: batch k+1's packing and H2D overlap k
            cs.submit_packed(b, now, nold)
            if j >= 1:
                cs.wait()
        cs.wait()
        t_pipe = time.perf_counter() - t0
        T0 = host[0][0].T
        pcie = {"serial": round(n * T0 / t_serial, 1), "pipelined": round(n * T0 / t_pipe, 1), "unit": "txn/s",
                "batches": n, "host_bytes_per_batch": int(np.mean([b.nbytes() for b, _n, _o in host])),
                "path": "host SoA batch -> pinned staging -> H2D -> detectConflicts pipeline -> verdict D2H "
                        "(fdbcs_batch_detect_packed; pipelined: fdbcs_batch_submit_packed / fdbcs_batch_wait)"}
        del host

    # ---- Resolver load metrics (not `value`): iopsSample roll of whole batches on the device ----
    lm = None
    if mode == "single" and args.lm_batches > 0:
        from foundationdb_amd.load_metrics import KEY_BYTES_PER_SAMPLE, SAMPLE_EXPIRATION_TIME, IopsSample
        smp = IopsSample(KEY_BYTES_PER_SAMPLE, seed=1)
        first = args.warmup + n_stage + 2 * args.pcie_batches + 2
        t_add, sampled, n_rng = 0.0, 0, 0
        for j in range(args.lm_batches):
            b, now, nold = src.wl.batch(first + j)
            cs.detect_packed(b, now, nold)  # (untimed) leaves the batch in HBM for the roll
            t0 = time.perf_counter()
            sampled += smp.add_batch(cs, j * 0.01 + SAMPLE_EXPIRATION_TIME)
            t_add += time.perf_counter() - t0
            n_rng += b.R + b.W
            smp.poll(j * 0.01)
        lm = {"us_per_batch": round(t_add / args.lm_batches * 1e6, 2), "ranges_per_batch": n_rng // args.lm_batches,
              "sampled_per_batch": round(sampled / args.lm_batches, 1), "sample_size": smp.size(),
              "units_per_sample": KEY_BYTES_PER_SAMPLE, "batches": args.lm_batches,
              "path": "fdbcs_sample_add_batch on the batch resident in HBM: device roll + ordered compaction + key "
                      "gather written to pinned host memory, host sample insert (synchronous wall time)"}
        smp.close()

    # ---- CPU baseline (oracle, 1 core) on the same batches, same start state -----
    cpu = None
    if snap is not None:
        from oracle import CpuSpec
        vers, lens, offs, kb, v0, oldest, rk = snap
        c = CpuSpec()
        c.load_history_arrays(len(vers), vers, lens, offs, kb, v0=v0, oldest=oldest, removal_key=rk)
        n, mism, tc = 0, 0, 0.0
        gv = sub_verdicts.cpu().numpy()
        while n < args.steps and tc < args.cpu_seconds:
            b, now, nold = src.wl.batch(args.warmup + n)
            ts = time.perf_counter()
            vc = c.detect_packed(b, now, nold)
            tc += time.perf_counter() - ts
            mism += int((vc != gv[n][:b.T]).sum())
            n += 1
        cpu = {"value": round(n * Tg / tc, 1), "unit": "txn/s", "cores": 1, "kind": "port",
               "sample": f"config {cfg}: batches {args.warmup}..{args.warmup + n - 1} ({n} x {Tg} txns) from the "
                         f"GPU's steady-state history (H={H_pre}); verdict mismatches vs GPU: {mism}"}

    if rank == 0:
        if mode == "exact":
            how = ("protocol B: each GPU receives only the ranges intersecting its keys; RCCL MAX all-reduce of "
                   "conflict flags + all-gather of overlap edges + all-gather for the compaction window"
                   if sparse else
                   "protocol A: every GPU receives the whole batch; RCCL MAX all-reduce of conflict flags + "
                   "all-gather for the compaction window")
            workload = (f"config{cfg}: {Tg}-txn global batches ({args.txns}/GPU), {CONFIG_SHAPE.get(cfg, '')}, "
                        f"5M-version window; one exact resolver sharded by key range over {world} GPUs ({how})")
        elif mode == "resolvers":
            workload = (f"config{cfg}: {Tg}-txn global batches ({args.txns}/GPU), 5R+2W, uniform 16-byte keys, "
                        f"5M-version window; {world} key-range resolvers (proxy split + RCCL MIN combine)")
        else:
            workload = f"config{cfg}: {Tg}-txn batches, {CONFIG_SHAPE.get(cfg, '')}, 5M-version window"
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
            "config": {"workload": workload, "txns_per_batch": Tg, "history_pre": H_pre, "history_post": H_post,
                       "parallelism": {"exact": f"sharded{world}", "resolvers": f"keyrange{world}"}.get(mode, "single")},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
            "load_metrics": lm,
        }
        if alt:
            out["alt_modes"] = alt
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
