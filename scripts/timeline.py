"""One batch's device timeline from a rocprofv3 kernel + memory-copy trace.

usage: python scripts/timeline.py DIR [marker=k_unpack] [which=-5]
"""
import csv
import os
import sys


def main():
    d = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_unpack"
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -5
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fdbcs_dev::", "")[:30]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    mp = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(mp):
        for r in csv.DictReader(open(mp)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r["Direction"].replace("MEMORY_COPY_", "")))
    ev.sort()
    idx = [i for i, e in enumerate(ev) if e[2].startswith(marker)]
    i0, i1 = idx[which], idx[which + 1]
    t0 = ev[i0][0]
    for e in ev[max(0, i0 - 6):i1 + 1]:
        print(f"{(e[0] - t0) / 1e3:9.1f} {(e[1] - t0) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:7.1f}  {e[2]}")


if __name__ == "__main__":
    main()
