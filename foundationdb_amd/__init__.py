"""MI355X-native FoundationDB Resolver conflict set (ConflictSet.h over HIP).

Public surface (mirrors fdbserver/ConflictSet.h):
    ConflictSet, ConflictBatch, CONFLICT / TOO_OLD / COMMITTED, FdbcsError
plus PackedBatch (whole-batch entry) and Workload (synthetic batches).
"""
from ._abi import COMMITTED, CONFLICT, TOO_OLD, FdbcsError  # noqa: F401
from .batch import PackedBatch  # noqa: F401
from .conflict_set import ConflictBatch, ConflictSet  # noqa: F401

__all__ = ["ConflictSet", "ConflictBatch", "PackedBatch", "FdbcsError", "CONFLICT", "TOO_OLD", "COMMITTED"]
