"""Generate the stream fixtures of SURVEY.md §8c (2-5) from the native
generator and the CPU restatement (oracle/cpu_spec.cpp).

    python tests/golden/make_streams.py            # all
    python tests/golden/make_streams.py config2    # one

Each fixture pins, per batch: a SHA-256 of the generated input (so a change
of the generator is caught, not silently re-baselined), the verdicts (2 bits
per transaction, base64), the verdict counts, and the history after the
batch as H, a SHA-256 of its canonical serialization (streams.py) and 32
sampled boundaries, plus removalKey / oldestVersion.

Provenance: oracle/cpu_spec.cpp, the build's restatement of SURVEY.md
Appendix A, itself checked against oracle/spec.py and the small fixtures.
The reference engine cannot be executed here: "parity
unpinned" -- these vectors pin the GPU engine and the restatement to each
other at realistic sizes.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from golden.streams import STREAMS, batch_sha, history_record, pack_verdicts  # noqa: E402


def make(name):
    from foundationdb_amd.workload import Workload
    from oracle import CpuSpec

    spec = STREAMS[name]
    wl = Workload(spec["config"], txns=spec["txns"])
    cs = CpuSpec()
    if spec["config"] == 4:  # wide reads end at the S-th boundary after their begin
        wl.set_successor(cs)
    out = []
    t0 = time.time()
    for i in range(spec.get("prefill", 0)):  # unrecorded batches [0, prefill) from an empty history
        b, now, nold = wl.batch(i)
        cs.detect_packed(b, now, nold)
        if i % 250 == 0:
            print(f"{name}: prefill batch {i}, {time.time() - t0:.0f}s", flush=True)
    for i in range(spec["first"], spec["first"] + spec["batches"]):
        b, now, nold = wl.batch(i)
        v = cs.detect_packed(b, now, nold)
        rec = {"index": i, "now": now, "new_oldest": nold, "input_sha256": batch_sha(b),
               "verdict_counts": [int((v == k).sum()) for k in range(3)], "verdict_b64": pack_verdicts(v)}
        rec.update(history_record(cs))
        out.append(rec)
    cs.close()
    wl.close()
    path = os.path.join(HERE, f"stream_{name}.json")
    with open(path, "w") as f:
        json.dump({"source": "oracle/cpu_spec.cpp (SURVEY.md Appendix A restatement); parity unpinned",
                   "generator": "foundationdb_amd/csrc/workload.cpp (fdbwl_generate, SURVEY.md §8d)",
                   "stream": name, **spec, "batches_out": out}, f, separators=(",", ":"))
    print(f"{path}: {len(out)} batches, H={out[-1]['H']}, {time.time() - t0:.1f}s")


if __name__ == "__main__":
    for n in (sys.argv[1:] or list(STREAMS)):
        make(n)
