"""Aggregate rocprofv3 --pmc counter CSVs per kernel over the last N batches.

usage: python scripts/pmc_summary.py gpurun_out/pmc [batches=50] [marker=k_ingest] [out.json] [history_pre]
Each pN/ directory holds one pass.  FETCH_SIZE is doubled (gfx950 reports half
of the bytes of wide coalesced reads: MI355X_MICROARCH.md §HBM); both
FETCH_SIZE and WRITE_SIZE are reported by rocprofv3 in KB.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(path):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def main():
    root = sys.argv[1]
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    marker = sys.argv[3] if len(sys.argv) > 3 else "k_ingest"
    per_kernel = defaultdict(lambda: defaultdict(float))
    for d in sorted(glob.glob(os.path.join(root, "p*"))):
        rows = load(d)
        if not rows:
            continue
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
        disp = sorted({int(r["Dispatch_Id"]) for r in rows})
        starts = sorted({int(r["Dispatch_Id"]) for r in rows if marker in r["Kernel_Name"]})
        first = starts[-nb] if len(starts) >= nb else starts[0]
        last = starts[-1]
        for r in rows:
            did = int(r["Dispatch_Id"])
            if not (first <= did < last):
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fdbcs_dev::", "")
            per_kernel[name][r["Counter_Name"]] += float(r["Counter_Value"])
    batches = nb - 1
    print(f"per batch (over {batches} batches); FETCH doubled per gfx950 correction; bytes")
    tot_f = tot_w = 0.0
    names = sorted(per_kernel, key=lambda k: -per_kernel[k].get("FETCH_SIZE", 0))
    for k in names:
        c = per_kernel[k]
        fb = 2 * c.get("FETCH_SIZE", 0) * 1024 / batches
        wb = c.get("WRITE_SIZE", 0) * 1024 / batches
        tot_f += fb
        tot_w += wb
        extra = " ".join(f"{n}={v / batches:.0f}" for n, v in sorted(c.items()) if n not in ("FETCH_SIZE", "WRITE_SIZE"))
        print(f"{k[:32]:32s} fetch {fb / 1e6:9.2f} MB  write {wb / 1e6:9.2f} MB  {extra}")
    print(f"TOTAL fetch {tot_f / 1e6:.2f} MB write {tot_w / 1e6:.2f} MB per batch -> {(tot_f + tot_w) / 1e6:.2f} MB")
    if len(sys.argv) > 4:  # JSON for bench.py's roofline.traffic
        import json
        with open(sys.argv[4], "w") as f:
            json.dump({"bytes_per_batch": round(tot_f + tot_w), "fetch_bytes": round(tot_f), "write_bytes": round(tot_w),
                       "batches": batches,
                       "history_pre": int(sys.argv[5]) if len(sys.argv) > 5 else None,
                       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over the bench workload; "
                                 "FETCH_SIZE x2 (gfx950 correction), KB->bytes; summed over all kernels of a batch",
                       "per_kernel_bytes": {k: round(2 * per_kernel[k].get("FETCH_SIZE", 0) * 1024 / batches
                                                     + per_kernel[k].get("WRITE_SIZE", 0) * 1024 / batches)
                                            for k in names}}, f, indent=1)


if __name__ == "__main__":
    main()
