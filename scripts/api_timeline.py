"""Host + device timeline of the Resolver window from one rocprofv3 run with
--kernel-trace --hip-runtime-trace --memory-copy-trace over a bench run with
FDBWL_MARK=1 (workload.cpp trace_mark: hipPeekAtLastError at the window's
start, at the end of the adds and at detectConflicts' return).

usage: python scripts/api_timeline.py DIR [last=20] [show=2]
Prints per-batch phase averages over the last `last` windows and the full
event list (API calls on the bench thread, kernels, copies) of `show` of them,
times in us from the end of the adds.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def find(d, name):
    f = glob.glob(os.path.join(d, "**", f"*{name}"), recursive=True)
    return f[0] if f else None


def short(n):
    return n.split("(")[0].replace("void ", "").replace("fdbcs_dev::", "")[:34]


def load_db(path):
    """The same three record lists from a rocpd SQLite output (rocprofv3's
    default output format on this image)."""
    import sqlite3
    c = sqlite3.connect(path)
    api = [{"Function": n, "Thread_Id": str(t), "Start_Timestamp": s, "End_Timestamp": e}
           for n, t, s, e in c.execute("select name, tid, start, end from regions")]
    ker = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
           for n, s, e in c.execute("select name, start, end from kernels")]
    cp = [{"Direction": n, "Bytes": b, "Start_Timestamp": s, "End_Timestamp": e}
          for n, b, s, e in c.execute("select name, size, start, end from memory_copies")]
    return api, ker, cp


def main():
    d = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    show = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    db = find(d, "_results.db")
    if db:
        api, ker, cps = load_db(db)
    else:
        api = list(csv.DictReader(open(find(d, "hip_api_trace.csv"))))
        ker = list(csv.DictReader(open(find(d, "kernel_trace.csv"))))
        mp = find(d, "memory_copy_trace.csv")
        cps = list(csv.DictReader(open(mp))) if mp else []
    marks = sorted(int(r["Start_Timestamp"]) for r in api if r["Function"] == "hipPeekAtLastError")
    tid = defaultdict(int)
    for r in api:
        if r["Function"] == "hipPeekAtLastError":
            tid[r["Thread_Id"]] += 1
    main_tid = max(tid, key=tid.get)
    calls = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api " + r["Function"]) for r in api
                   if r["Thread_Id"] == main_tid and r["Function"] != "hipPeekAtLastError")
    dev = []
    for r in ker:
        dev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + short(r["Kernel_Name"])))
    for r in cps:
        dev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    "C " + r["Direction"].replace("MEMORY_COPY_", "") + f" {int(r.get('Bytes', 0) or 0) // 1024}K"))
    dev.sort()
    n = len(marks) // 3
    wins = [(marks[3 * i], marks[3 * i + 1], marks[3 * i + 2]) for i in range(n)][-last:]
    agg = defaultdict(list)
    for k, (t0, ta, t1) in enumerate(wins):
        agg["window"].append(t1 - t0)
        agg["adds"].append(ta - t0)
        agg["detect"].append(t1 - ta)
        ev = [e for e in dev if ta - 400_000 <= e[0] <= t1]
        ks = [e for e in ev if e[2].startswith("K ") and e[0] >= ta - 50_000]
        ing = [e for e in ks if "ingest" in e[2] and e[0] >= ta]
        live = [e for e in ev if "k_live_ingest" in e[2] and e[0] <= ta]
        if live:  # (live ingest: the kernel began at fdbcs_batch_begin, before the adds ended)
            agg["live_ingest_end-adds_end"].append(live[-1][1] - ta)
            agg["live_ingest_start-window_start"].append(live[-1][0] - t0)
        dec = [e for e in ks if "decide" in e[2] and e[0] >= ta]
        cps = [e for e in ev if e[2].startswith("C HOST_TO_DEVICE") and e[0] <= (ing[0][0] if ing else t1)]
        prev_end = max((e[1] for e in dev if e[1] <= (ing[0][0] if ing else t1) and e[2].startswith("K ")), default=None)
        if ing:
            agg["adds_end->ingest_start"].append(ing[0][0] - ta)
            agg["prev_batch_last_kernel_end->ingest_start"].append(ing[0][0] - prev_end if prev_end else 0)
            if cps:
                agg["last_copy_start-adds_end"].append(cps[-1][0] - ta)
                agg["last_copy_dur"].append(cps[-1][1] - cps[-1][0])
                agg["last_copy_end->ingest_start"].append(ing[0][0] - cps[-1][1])
            if dec:
                agg["ingest_start->decide_start"].append(dec[0][0] - ing[0][0])
                agg["decide_start->detect_return"].append(t1 - dec[0][0])
        cs = [c for c in calls if ta <= c[0] <= t1]
        agg["api_calls_in_detect"].append(len(cs) * 1000)
        agg["api_time_in_detect"].append(sum(c[1] - c[0] for c in cs))
        if k >= len(wins) - show:
            print(f"--- window {k}: adds {(ta - t0) / 1e3:.1f} us, detect {(t1 - ta) / 1e3:.1f} us (times from adds end)")
            both = sorted([c for c in calls if t0 <= c[0] <= t1] + [e for e in dev if t0 - 50_000 <= e[0] <= t1 + 50_000])
            for e in both:
                print(f"{(e[0] - ta) / 1e3:9.1f} {(e[1] - ta) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:7.1f}  {e[2]}")
    print(f"=== averages over {len(wins)} windows (us)")
    for k, v in agg.items():
        v = sorted(v)
        print(f"{k:45s} mean {sum(v) / len(v) / 1e3:8.1f}  p50 {v[len(v) // 2] / 1e3:8.1f}  max {v[-1] / 1e3:8.1f}")


if __name__ == "__main__":
    main()
