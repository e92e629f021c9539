"""Summarize a rocprofv3 kernel trace over the last N batches (the bench's timed region).

usage: python scripts/prof_summary.py run_kernel_trace.csv [last_batches=200] [marker=k_prep]
Each batch starts with one launch of `marker`; per-kernel averages are taken
over the launches that belong to the last N batches only (warmup excluded).
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    marker = sys.argv[3] if len(sys.argv) > 3 else "k_ingest"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    last = min(last, len(starts))
    first = starts[-last]
    sel = rows[first:starts[-1]]  # whole batches only (the last one is partial)
    nb = last - 1
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in sel:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fdbcs_dev::", "")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[name] += d
        cnt[name] += 1
    span = (int(rows[starts[-1]]["Start_Timestamp"]) - int(rows[first]["Start_Timestamp"])) / 1e3 / nb
    busy = sum(tot.values()) / nb
    print(f"batches {nb}: span {span:.1f} us/batch, kernel-busy {busy:.1f} us/batch, gaps {span - busy:.1f} us")
    print(f"{'kernel':40s} {'calls/b':>8s} {'avg us':>8s} {'us/batch':>9s}")
    for k in sorted(tot, key=lambda k: -tot[k]):
        print(f"{k[:40]:40s} {cnt[k] / nb:8.2f} {tot[k] / cnt[k]:8.2f} {tot[k] / nb:9.2f}")


if __name__ == "__main__":
    main()
