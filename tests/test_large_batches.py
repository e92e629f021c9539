"""GPU parity of the large-batch path (T > 65,536: config 5's 1 M-txn batches).

Large batches sort their endpoints with a merge sort and keep overlap edges
undeduplicated (no T x T pair matrix), growing the edge list and searching
again when a batch overflows it (DESIGN.md §Large batches).  Verdicts and the
full history must equal the CPU oracle's, exactly as for small batches.

FDBCS_TEST_LARGE_BATCH forces the large path at small T so the golden and
random streams (empty keys, \\x00 keys, long-key tails, Zipf chains) run
through it; FDBCS_TEST_EDGE_CAP shrinks the first edge list so the overflow
path runs.
"""
import json
import os

import numpy as np
import pytest

from foundationdb_amd import ConflictSet
from foundationdb_amd.conflict_set import COMMITTED
from foundationdb_amd.batch import PackedBatch
from foundationdb_amd.workload import Workload
from gen import mixed_stream, tiny_stream
from oracle import CpuSpec

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def same_history(g, c):
    gv, gl, go, gk = g.dump_arrays()
    cv, cl, co, ck = c.dump_arrays()
    assert len(gv) == len(cv), (len(gv), len(cv))
    if len(gv) == 0:
        return
    assert np.array_equal(gv, cv), "versions differ"
    assert np.array_equal(gl, cl), "key lengths differ"
    n = int(gl.astype(np.int64).sum())
    assert np.array_equal(gk[:n], ck[:n]), "key bytes differ"


def check_pair(g, c, batch, now, nold, history=True):
    vg = g.detect_packed(batch, now, nold)
    vc = c.detect_packed(batch, now, nold)
    assert np.array_equal(vg, vc), (np.nonzero(vg != vc)[0][:10], vg[:20], vc[:20])
    assert g.oldest_version == c.oldest_version
    if history:
        same_history(g, c)
        assert g.removal_key() == c.removal_key()
    return vg


class forced:
    """Set test environment switches for the duration of a block."""

    def __init__(self, **env):
        self.env = env

    def __enter__(self):
        for k, v in self.env.items():
            os.environ[k] = v

    def __exit__(self, *a):
        for k in self.env:
            os.environ.pop(k, None)


@pytest.fixture()
def cs(gpu):
    g = ConflictSet()
    yield g
    g.close()


def test_forced_large_golden(cs):
    with forced(FDBCS_TEST_LARGE_BATCH="1"):
        for name in ["tiny_alphabet", "long_keys", "clear_mid_stream", "appendix_c"]:
            with open(os.path.join(GOLDEN, f"{name}.json")) as f:
                streams = json.load(f)["streams"]
            for stream in streams:
                cs.clear(0)
                cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
                for e in stream:
                    if "clear_before" in e:
                        cs.clear(e["clear_before"])
                    txns = [(s, [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in r],
                             [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in w]) for s, r, w in e["txns"]]
                    v = cs.detect_packed(PackedBatch.from_txns(txns), e["now"], e["new_oldest"])
                    assert list(v) == e["verdict"], name
                    assert [[k.hex(), ver] for k, ver in cs.history()] == e["history"], name
                    assert cs.removal_key().hex() == e["removal_key"], name


@pytest.mark.parametrize("maxlen", [3, 40])
def test_forced_large_tiny_streams(cs, maxlen):
    with forced(FDBCS_TEST_LARGE_BATCH="1"):
        for seed in range(10):
            cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
            c = CpuSpec()
            for batch, now, nold in tiny_stream(seed * 7 + maxlen, n_batches=20, maxlen=maxlen):
                check_pair(cs, c, batch, now, nold)


def test_forced_large_mixed_streams(cs):
    with forced(FDBCS_TEST_LARGE_BATCH="1"):
        for seed in range(3):
            cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
            c = CpuSpec()
            for batch, now, nold in mixed_stream(100 + seed, n_batches=10, max_txns=1500, keyspace=4000):
                check_pair(cs, c, batch, now, nold)


@pytest.mark.parametrize("cfg,T,nb", [(2, 3000, 6), (3, 3000, 6), (4, 1500, 5)])
def test_forced_large_workloads(cs, cfg, T, nb):
    """Merge passes over several tiles (R = 5T read begins), Zipf duplicates
    and chains (config 3), 68-100-byte keys compared through their tails
    (config 4); the small path resumes afterwards from the large path's
    quantiles."""
    c = CpuSpec()
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    wl = Workload(cfg, txns=T)
    with forced(FDBCS_TEST_LARGE_BATCH="1"):
        for i in range(nb):
            batch, now, nold = wl.batch(i)
            check_pair(cs, c, batch, now, nold, history=(i % 2 == 1 or i == nb - 1))
    for i in range(nb, nb + 3):  # back on the sample sort, splitting by the merge sort's quantiles
        batch, now, nold = wl.batch(i)
        check_pair(cs, c, batch, now, nold)


def test_edge_list_overflow_regrows(gpu):
    """Zipf batches produce thousands of overlap pairs; a 16-entry first edge
    list overflows, is grown to the count and searched again."""
    with forced(FDBCS_TEST_LARGE_BATCH="1", FDBCS_TEST_EDGE_CAP="16"):
        g = ConflictSet()
        try:
            c = CpuSpec()
            wl = Workload(3, txns=2000)
            for i in range(4):
                batch, now, nold = wl.batch(i)
                check_pair(g, c, batch, now, nold)
        finally:
            g.close()


@pytest.mark.parametrize("cfg,T,nb", [(2, 100_000, 3), (1, 80_000, 3)])
def test_real_large_batches(cs, cfg, T, nb):
    """T past LARGE_T with no forcing: 500 K read begins and 400 K write
    endpoints per batch (config 2 shape), and skipListTest's dense 2*10^7-key
    space with short ranges (config 1 shape: thousands of overlap edges)."""
    c = CpuSpec()
    cs.load_history([], [], v0=0, oldest=0, removal_key=b"")
    wl = Workload(cfg, txns=T)
    for i in range(nb):
        batch, now, nold = wl.batch(i)
        check_pair(cs, c, batch, now, nold, history=(i == nb - 1))


def test_config5_one_gpu_share(gpu):
    """Config 5 at one GPU's share: 10^8 history
    boundaries over 8 GPUs is 12.5 M per GPU, and in exact mode A every GPU
    resolves the whole 10^6-txn batch against its part.  Preload 7 blind-write
    batches of 10^6 point writes (bench.py's config-5 preload, ~14 M
    boundaries), load the oracle from the GPU's own dump, then three full
    10^6-txn config-5 batches: verdicts, oldest version and the whole history
    after the last batch must be identical."""
    g = ConflictSet(device=0, max_history=30_000_000)
    c = CpuSpec()
    try:
        Workload(50, txns=1_000_000).prefill(g, 0, 7)
        vers, lens, offs, kb = g.dump_arrays()
        assert len(vers) > 12_000_000, len(vers)
        c.load_history_arrays(len(vers), vers, lens, offs, kb, v0=g.header_version, oldest=g.oldest_version,
                              removal_key=g.removal_key())
        del vers, lens, offs, kb
        same_history(g, c)
        wl = Workload(5, txns=1_000_000)
        for i in range(3):
            batch, now, nold = wl.batch(i)
            vg = check_pair(g, c, batch, now, nold, history=(i == 2))
            assert (vg == COMMITTED).any()
    finally:
        c.close()
        g.close()
