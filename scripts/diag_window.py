"""Per-batch Resolver-window timings (adds / detect) over repeated runs of K
batches after the bench's steady-state prefill -- to find transients in the
driver's 20-batch timed region.  Diagnostic, not the bench.

usage: python scripts/diag_window.py [rounds=6] [steps=20] [pin=none|numa|core]
  pin=numa: the process on the CPUs of the GPU's NUMA node (within its affinity)
  pin=core: one CPU of those
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def gpu_numa_cpus():
    import glob
    allowed = os.sched_getaffinity(0)
    for d in glob.glob("/sys/class/drm/card*/device/numa_node"):
        try:
            node = int(open(d).read())
        except (OSError, ValueError):
            continue
        if node < 0:
            continue
        cl = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
        cpus = set()
        for part in cl.split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        both = sorted(cpus & allowed)
        if both:
            return node, both
    return None, sorted(allowed)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    pin = sys.argv[3] if len(sys.argv) > 3 else "none"
    node, cpus = gpu_numa_cpus()
    print(f"# affinity {len(os.sched_getaffinity(0))} cpus; gpu numa node {node}: {len(cpus)} of them", flush=True)
    if pin == "numa":
        os.sched_setaffinity(0, cpus)
    elif pin == "core":
        os.sched_setaffinity(0, cpus[:1])
    import torch
    torch.cuda.set_device(0)
    from foundationdb_amd import ConflictSet
    from foundationdb_amd.workload import Workload
    wl = Workload(2, txns=5000)
    cs = ConflictSet(device=0, max_history=30_000_000)
    wl.prefill(cs, 0, 2500)
    first = 2500
    for r in range(rounds):
        run = wl.prepare_run(first, steps)
        us, add, _v = run.run(cs, verdicts=False)
        del run
        first += steps
        print(f"round {r}: window mean {us.mean():7.1f} p50 {np.median(us):7.1f} max {us.max():7.1f} | adds mean "
              f"{add.mean():7.1f} p50 {np.median(add):7.1f} | detect p50 {np.median(us - add):6.1f}", flush=True)
        print("   windows", " ".join(f"{x:.0f}" for x in us), flush=True)
        print("   adds   ", " ".join(f"{x:.0f}" for x in add), flush=True)
        time.sleep(0.2)
    cs.close()


if __name__ == "__main__":
    main()
