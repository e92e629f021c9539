"""Stream fixtures: definitions and the canonical forms
shared by tests/golden/make_streams.py and the tests that replay them."""
import base64
import hashlib
import struct

import numpy as np

# name -> generator config, transactions per batch, first batch index, batches
STREAMS = {
    # 2. skipListTest-like: 2,500 txns, 1R+1W, setK keys (SkipList.cpp:1436-1486)
    "skiplisttest": {"config": 1, "txns": 0, "first": 0, "batches": 20},
    # 3. config 2 from an empty history: uniform 16-byte keys, 5R+2W
    "config2": {"config": 2, "txns": 0, "first": 0, "batches": 50},
    # 4. config 3: Zipf(0.99) hot keys, long intra-batch chains
    "config3": {"config": 3, "txns": 0, "first": 0, "batches": 20},
    # 5. config 4: 68-100-byte keys over 16 tenants (tails past byte 17)
    "config4": {"config": 4, "txns": 0, "first": 0, "batches": 20},
    # 6. config 2 at the bench's steady state: batches 2,500-2,519 after 2,500
    #    unrecorded batches from an empty history (H ~ 19 M, compaction active;
    #    VERDICT r04 item 1) -- only the recorded batches' inputs are hashed
    "config2_steady": {"config": 2, "txns": 0, "first": 2500, "batches": 20, "prefill": 2500},
}
N_SAMPLES = 32


def batch_sha(b):
    """SHA-256 of a PackedBatch: a tag, snapshots, per-txn range offsets,
    every key slot's length (u32 LE), then the slots' bytes in slot order."""
    h = hashlib.sha256(b"fdbcs-batch-v1")
    h.update(np.ascontiguousarray(b.snapshot, np.int64).astype("<i8").tobytes())
    h.update(np.ascontiguousarray(b.read_off, np.int32).astype("<i4").tobytes())
    h.update(np.ascontiguousarray(b.write_off, np.int32).astype("<i4").tobytes())
    lens = np.asarray(b.key_len, np.int64)
    h.update(lens.astype("<u4").tobytes())
    total = int(lens.sum())
    if total:
        start = np.cumsum(lens) - lens
        pos = np.repeat(np.asarray(b.key_off, np.int64) - start, lens) + np.arange(total)
        h.update(np.asarray(b.key_bytes, np.uint8)[pos].tobytes())
    return h.hexdigest()


def pack_verdicts(v):
    """Verdict bytes (0/1/2) as 2 bits each, little-endian within a byte, base64."""
    v = np.asarray(v, np.uint8)
    pad = (-len(v)) % 4
    w = np.concatenate([v, np.zeros(pad, np.uint8)]).reshape(-1, 4)
    packed = (w[:, 0] | (w[:, 1] << 2) | (w[:, 2] << 4) | (w[:, 3] << 6)).astype(np.uint8)
    return base64.b64encode(packed.tobytes()).decode()


def unpack_verdicts(s, n):
    p = np.frombuffer(base64.b64decode(s), np.uint8)
    v = np.stack([(p >> (2 * k)) & 3 for k in range(4)], axis=1).reshape(-1)
    return v[:n].astype(np.uint8)


def history_sha(vers, lens, offs, kb):
    """SHA-256 of the boundary list in order: a tag, every key length (u32
    LE), every key's bytes concatenated in order, every version (i64 LE)."""
    lens = np.asarray(lens, np.int64)
    offs = np.asarray(offs, np.int64)
    kb = np.asarray(kb, np.uint8)
    h = hashlib.sha256(b"fdbcs-history-v1")
    h.update(lens.astype("<u4").tobytes())
    total = int(lens.sum())
    if total:
        start = np.cumsum(lens) - lens  # position of each key in the concatenation
        if np.array_equal(offs - start, np.full_like(offs, offs[0])):  # (packed in order: one slice)
            h.update(kb[int(offs[0]):int(offs[0]) + total].tobytes())
        else:
            pos = np.repeat(offs - start, lens) + np.arange(total)
            h.update(kb[pos].tobytes())
    h.update(np.asarray(vers, np.int64).astype("<i8").tobytes())
    return h.hexdigest()


def history_record(cs):
    """The post-batch state of a conflict set (ConflictSet or CpuSpec) in
    fixture form."""
    vers, lens, offs, kb = cs.dump_arrays()
    H = int(len(vers))
    kb = np.asarray(kb, np.uint8)
    samples = []
    for j in range(N_SAMPLES if H else 0):
        i = j * H // N_SAMPLES
        o, n = int(offs[i]), int(lens[i])
        samples.append([i, kb[o:o + n].tobytes().hex(), int(vers[i])])
    def val(x):
        return x() if callable(x) else x
    return {"H": H, "history_sha256": history_sha(vers, lens, offs, kb), "samples": samples,
            "removal_key": cs.removal_key().hex(), "oldest": int(val(cs.oldest_version)),
            "v0": int(val(cs.header_version))}
