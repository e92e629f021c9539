"""CPU: the oracle restatements agree with each other and with the golden fixtures."""
import json
import os

import pytest

from foundationdb_amd.batch import PackedBatch
from gen import mixed_stream, tiny_stream
from oracle import CpuSpec, SpecBatch, SpecConflictSet, spec_detect

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixture(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)["streams"]


def fixture_batches(stream):
    for e in stream:
        txns = [(snap, [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in r],
                 [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in w]) for snap, r, w in e["txns"]]
        yield e, PackedBatch.from_txns(txns)


FIXTURES = ["tiny_alphabet", "long_keys", "clear_mid_stream", "appendix_c"]


@pytest.mark.parametrize("name", FIXTURES)
def test_cpu_spec_reproduces_golden(name):
    for stream in load_fixture(name):
        cs = CpuSpec()
        for e, batch in fixture_batches(stream):
            if "clear_before" in e:
                cs.clear(e["clear_before"])
            v = cs.detect_packed(batch, e["now"], e["new_oldest"])
            assert list(v) == e["verdict"]
            assert [(k.hex(), ver) for k, ver in cs.history()] == [tuple(x) for x in e["history"]]
            assert cs.removal_key().hex() == e["removal_key"]
            assert cs.oldest_version == e["oldest"]
            assert cs.header_version == e["v0"]


@pytest.mark.parametrize("name", FIXTURES)
def test_python_spec_reproduces_golden(name):
    for stream in load_fixture(name):
        cs = SpecConflictSet()
        for e, batch in fixture_batches(stream):
            if "clear_before" in e:
                cs.clear(e["clear_before"])
            assert spec_detect(cs, batch, e["now"], e["new_oldest"]) == e["verdict"]
            assert [[k.hex(), v] for k, v in cs.history()] == e["history"]


@pytest.mark.parametrize("maxlen", [3, 11, 30])
def test_cpu_spec_matches_python_spec_tiny(maxlen):
    for seed in range(40):
        spec, cpu = SpecConflictSet(), CpuSpec()
        for batch, now, nold in tiny_stream(seed * 31 + maxlen, n_batches=25, maxlen=maxlen):
            assert list(cpu.detect_packed(batch, now, nold)) == spec_detect(spec, batch, now, nold)
            assert cpu.history() == spec.history()
            assert cpu.removal_key() == spec.removal_key
            assert cpu.oldest_version == spec.oldest


def test_cpu_spec_matches_python_spec_mixed():
    for seed in range(3):
        spec, cpu = SpecConflictSet(), CpuSpec()
        for batch, now, nold in mixed_stream(seed, n_batches=10):
            assert list(cpu.detect_packed(batch, now, nold)) == spec_detect(spec, batch, now, nold)
            assert cpu.history() == spec.history()
            assert cpu.removal_key() == spec.removal_key


def test_spec_api_appends_like_reference():
    """nonConflicting / tooOld are appended to, never cleared (SkipList.cpp:1188-1194)."""
    cs = SpecConflictSet()
    b = SpecBatch(cs)
    b.add_transaction([], [(b"a", b"b")], 0)
    v, nc, to = b.detect_conflicts(10, 5)
    assert v == [2] and nc == [0] and to == []
    b = SpecBatch(cs)
    b.add_transaction([(b"a", b"b")], [], 1)   # snapshot 1 < oldest 5 with a read: tooOld
    b.add_transaction([(b"a", b"b")], [], 10)  # sees a@10, 10 > 10 is false: commits
    b.add_transaction([], [(b"c", b"d")], 1)   # no reads: never tooOld
    v, nc, to = b.detect_conflicts(20, 5)
    assert v == [1, 2, 2] and nc == [1, 2] and to == [0]


def test_empty_range_rejected():
    cs = SpecConflictSet()
    b = SpecBatch(cs)
    with pytest.raises(AssertionError):
        b.add_transaction([(b"a", b"a")], [], 0)
