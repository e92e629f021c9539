"""Stream fixtures (tests/golden/stream_*.json) replayed.

CPU: the generator still produces the recorded inputs (every batch's input
SHA-256) and the CPU restatement reproduces the recorded verdicts and
post-batch histories on a prefix of each stream.  GPU: the whole stream
through the engine -- configs 2, 3 and 4 through the Resolver's per-transaction
loop (fdbwl_run_resolver: fdbcs_batch_begin / add / detect), the others as
packed batches -- bit-exact after every batch: verdicts, H, the history's
SHA-256, 32 sampled boundaries, removalKey, oldestVersion.
"""
import json
import os

import numpy as np
import pytest

from golden.streams import STREAMS, batch_sha, history_record, unpack_verdicts

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CPU_PREFIX = {"skiplisttest": 20, "config2": 8, "config3": 20, "config4": 20, "config2_steady": 0}


def load(name):
    with open(os.path.join(GOLDEN, f"stream_{name}.json")) as f:
        return json.load(f)


def check_record(got, want, name, i):
    for k in ("H", "history_sha256", "removal_key", "oldest", "v0"):
        assert got[k] == want[k], f"{name} batch {i}: {k} {got[k]} != {want[k]}"
    assert got["samples"] == want["samples"], f"{name} batch {i}: sampled boundaries differ"


@pytest.mark.parametrize("name", [n for n in STREAMS if STREAMS[n]["config"] != 4])
def test_generator_inputs_unchanged(name):
    """(config 4's inputs depend on the history: checked by the replays below)"""
    from foundationdb_amd.workload import Workload
    fx = load(name)
    wl = Workload(fx["config"], txns=fx["txns"])
    for rec in fx["batches_out"]:
        b, now, nold = wl.batch(rec["index"])
        assert (now, nold) == (rec["now"], rec["new_oldest"])
        assert batch_sha(b) == rec["input_sha256"], f"{name} batch {rec['index']}: generator output changed"
    wl.close()


@pytest.mark.parametrize("name", list(STREAMS))
def test_cpu_spec_reproduces_stream(name):
    from foundationdb_amd.workload import Workload
    from oracle import CpuSpec
    if not CPU_PREFIX[name]:
        pytest.skip("2,500 unrecorded batches first (~10 min of oracle time): made by make_streams.py, "
                    "replayed on the GPU only")
    fx = load(name)
    wl = Workload(fx["config"], txns=fx["txns"])
    cs = CpuSpec()
    if fx["config"] == 4:
        wl.set_successor(cs)
    for rec in fx["batches_out"][:CPU_PREFIX[name]]:
        b, now, nold = wl.batch(rec["index"])
        assert batch_sha(b) == rec["input_sha256"], f"{name} batch {rec['index']}: input differs"
        v = cs.detect_packed(b, now, nold)
        assert np.array_equal(v, unpack_verdicts(rec["verdict_b64"], b.T)), f"{name} batch {rec['index']}"
        check_record(history_record(cs), rec, name, rec["index"])
    cs.close()
    wl.close()


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", list(STREAMS))
def test_gpu_replays_stream(name):
    """config2_steady: batches 2,500-2,519 of config 2
    from an empty history -- the bench's steady state, H ~ 19 M, compaction
    sweeping -- checked against the oracle's own run (not the oracle loaded
    from the GPU's dump).  The first 2,500 go through the pipelined
    whole-batch path (fdbwl_prefill, as the bench's prefill), the recorded
    ones through the Resolver's loop, live from the second on."""
    from foundationdb_amd import ConflictSet
    from foundationdb_amd.workload import Workload
    fx = load(name)
    wl = Workload(fx["config"], txns=fx["txns"])
    prefill = fx.get("prefill", 0)
    cs = ConflictSet(device=0, max_history=24_000_000 if prefill else 4_000_000)
    if fx["config"] == 4:  # the wide reads' ends from the engine's own history (fdbcs_nth_after)
        wl.set_successor(cs)
    per_txn = name in ("config2", "config3", "config4", "config2_steady")  # (config 4: 68-100-byte keys)
    if prefill:
        wl.prefill(cs, 0, prefill)
    live0 = cs.batch_stats()["live_batches"]
    for rec in fx["batches_out"]:
        i = rec["index"]
        if per_txn:  # the Resolver's loop: begin, T x add, detect (native)
            run = wl.prepare_run(i, 1)
            _us, _add, v = run.run(cs, verdicts=True)
            v = v[0]
            del run
        else:
            b, now, nold = wl.batch(i)
            assert batch_sha(b) == rec["input_sha256"], f"{name} batch {i}: input differs"
            v = cs.detect_packed(b, now, nold)
        want = unpack_verdicts(rec["verdict_b64"], len(v))
        assert np.array_equal(np.asarray(v, np.uint8), want), \
            f"{name} batch {i}: {int((np.asarray(v) != want).sum())} verdicts differ"
        assert [int((np.asarray(v) == k).sum()) for k in range(3)] == rec["verdict_counts"]
        check_record(history_record(cs), rec, name, i)
    if prefill:  # every recorded batch after the first went through the live ingest
        assert cs.batch_stats()["live_batches"] - live0 == len(fx["batches_out"]) - 1, cs.batch_stats()
    cs.close()
    wl.close()
