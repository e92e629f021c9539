"""Debug helper: replay a golden fixture on the GPU and print the first mismatching batch."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from foundationdb_amd import ConflictSet  # noqa: E402
from foundationdb_amd.batch import PackedBatch  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "tiny_alphabet"
    cs = ConflictSet()
    streams = json.load(open(os.path.join(ROOT, "tests", "golden", f"{name}.json")))["streams"]
    for si, stream in enumerate(streams):
        cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
        prev = []
        for bi, e in enumerate(stream):
            if "clear_before" in e:
                cs.clear(e["clear_before"])
            txns = [(s, [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in r],
                     [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in w]) for s, r, w in e["txns"]]
            v = cs.detect_packed(PackedBatch.from_txns(txns), e["now"], e["new_oldest"])
            got = [[k.hex(), ver] for k, ver in cs.history()]
            if got != e["history"] or list(v) != e["verdict"]:
                print("stream", si, "batch", bi, "now", e["now"], "nold", e["new_oldest"])
                print("prev ", prev)
                print("got  ", got)
                print("want ", e["history"])
                print("verdict ok", list(v) == e["verdict"])
                for t, (s, r, w) in enumerate(txns):
                    print("  txn", t, s, [(a.hex(), b.hex()) for a, b in r], [(a.hex(), b.hex()) for a, b in w],
                          v[t])
                return
            prev = got
    print("all ok")


if __name__ == "__main__":
    main()
