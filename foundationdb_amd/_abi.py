"""ctypes mirror of include/fdbcs.h and the loader for the in-tree libraries.

The product library must be the HIP build: there is no CPU fallback.  Loading
fails loudly if ``libfdbcs.so`` is missing (run ``python -m
foundationdb_amd.build`` or ``__graft_entry__.build()``).
"""
import ctypes as C
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FDBCS_LIB_PATH", os.path.join(PKG, "libfdbcs.so"))  # override: experiments only
WL_PATH = os.path.join(PKG, "libfdbcs_workload.so")

CONFLICT, TOO_OLD, COMMITTED = 0, 1, 2

OK = 0
E_HIP, E_NOMEM, E_RANGE, E_STATE, E_ARG, E_KEY, E_NODEV, E_CAPACITY = -1, -2, -3, -4, -5, -6, -7, -8
MAX_KEY = 30001


class Range(C.Structure):
    _fields_ = [("begin", C.c_void_p), ("begin_len", C.c_uint32), ("end", C.c_void_p), ("end_len", C.c_uint32)]


class BatchView(C.Structure):
    _fields_ = [
        ("txn_count", C.c_int32),
        ("read_count", C.c_int32),
        ("write_count", C.c_int32),
        ("reserved", C.c_int32),
        ("snapshot", C.c_void_p),
        ("read_off", C.c_void_p),
        ("write_off", C.c_void_p),
        ("key_off", C.c_void_p),
        ("key_len", C.c_void_p),
        ("key_bytes", C.c_void_p),
        ("key_bytes_len", C.c_uint64),
    ]


class Config(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("flags", C.c_int32),  # FDBCS_BORROW_*
        ("max_history", C.c_int64),
        ("max_batch_keys", C.c_int64),
        ("tail_arena_bytes", C.c_int64),
    ]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.c_uint64)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint8), C.c_uint64)


class CommOps(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("allreduce_max_u8", ALLREDUCE_FN), ("allgather_u8", ALLGATHER_FN)]


COMM_ID_BYTES = 128

# (name, restype, argtypes) for every function declared in include/fdbcs.h
FDBCS_FUNCS = [
    ("fdbcs_create", C.c_int, [C.POINTER(C.c_void_p), C.c_int64, C.POINTER(Config)]),
    ("fdbcs_clear", C.c_int, [C.c_void_p, C.c_int64]),
    ("fdbcs_set_version", C.c_int, [C.c_void_p, C.c_int64]),
    ("fdbcs_destroy", None, [C.c_void_p]),
    ("fdbcs_batch_begin", C.c_int, [C.c_void_p]),
    ("fdbcs_batch_skip", C.c_int, [C.c_void_p, C.c_int32]),
    ("fdbcs_batch_add", C.c_int, [C.c_void_p, C.c_int64, C.POINTER(Range), C.c_int32, C.POINTER(Range), C.c_int32]),
    ("fdbcs_batch_detect", C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]),
    ("fdbcs_batch_txn_count", C.c_int32, [C.c_void_p]),
    ("fdbcs_batch_detect_packed", C.c_int, [C.c_void_p, C.POINTER(BatchView), C.c_int64, C.c_int64, C.c_void_p]),
    ("fdbcs_batch_submit_packed", C.c_int, [C.c_void_p, C.POINTER(BatchView), C.c_int64, C.c_int64]),
    ("fdbcs_batch_wait", C.c_int, [C.c_void_p, C.c_void_p]),
    ("fdbcs_detect_device", C.c_int, [C.c_void_p, C.POINTER(BatchView), C.c_int64, C.c_int64, C.c_void_p, C.c_int]),
    ("fdbcs_history_size", C.c_int64, [C.c_void_p]),
    ("fdbcs_header_version", C.c_int64, [C.c_void_p]),
    ("fdbcs_oldest_version", C.c_int64, [C.c_void_p]),
    ("fdbcs_dump_history", C.c_int64,
     [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    ("fdbcs_load_history", C.c_int,
     [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p,
      C.c_uint32]),
    ("fdbcs_removal_key", C.c_int32, [C.c_void_p, C.c_void_p, C.c_int32]),
    ("fdbcs_enable_stage_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("fdbcs_stage_times", C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_int]),
    ("fdbcs_stream", C.c_void_p, [C.c_void_p]),
    ("fdbcs_batch_stats", C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_int]),
    ("fdbcs_batch_refused_txn", C.c_int64, [C.c_void_p]),
    ("fdbcs_debug_phases", C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_int]),
    ("fdbcs_debug_prefix_skips", C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_int]),
    ("fdbcs_split_batch", C.c_int,
     [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(BatchView), C.c_void_p,
      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fdbcs_split_batch_keep_all", C.c_int,
     [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(BatchView), C.c_void_p,
      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fdbcs_key_owner", C.c_int32, [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]),
    ("fdbcs_scatter_verdicts", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    ("fdbcs_set_shard", C.c_int, [C.c_void_p, C.c_char_p, C.c_uint32, C.c_int, C.c_char_p, C.c_uint32, C.c_int]),
    ("fdbcs_shard_check", C.c_int, [C.c_void_p, C.POINTER(BatchView), C.c_int64, C.c_int64, C.c_int64, C.c_void_p]),
    ("fdbcs_shard_apply", C.c_int, [C.c_void_p, C.POINTER(BatchView), C.c_int64, C.c_int64, C.c_int64, C.c_char_p,
                                    C.c_int32, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64)]),
    ("fdbcs_shard_compact", C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_int64, C.c_int64, C.c_int64,
                                      C.c_void_p, C.c_int32, C.POINTER(C.c_int64)]),
    ("fdbcs_shard_set_protocol", C.c_int, [C.c_void_p, C.c_int]),
    ("fdbcs_shard_edge_count", C.c_int64, [C.c_void_p]),
    ("fdbcs_shard_get_edges", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]),
    ("fdbcs_shard_set_edges", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]),
    ("fdbcs_last_device_batch", C.c_int, [C.c_void_p, C.POINTER(BatchView)]),
    ("fdbcs_sample_create", C.c_int, [C.POINTER(C.c_void_p), C.c_int64, C.c_uint64]),
    ("fdbcs_sample_destroy", None, [C.c_void_p]),
    ("fdbcs_sample_add_batch", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(BatchView), C.c_int64, C.c_double,
                                         C.POINTER(C.c_int64)]),
    ("fdbcs_sample_add_metric", C.c_int, [C.c_void_p, C.c_char_p, C.c_uint32, C.c_int64]),
    ("fdbcs_sample_poll", C.c_int, [C.c_void_p, C.c_double]),
    ("fdbcs_sample_estimate", C.c_int64, [C.c_void_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32]),
    ("fdbcs_sample_split", C.c_int32, [C.c_void_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_int64,
                                       C.c_int, C.c_void_p, C.c_uint32]),
    ("fdbcs_sample_size", C.c_int64, [C.c_void_p]),
    ("fdbcs_sample_queue_size", C.c_int64, [C.c_void_p]),
    ("fdbcs_sample_entry", C.c_int32, [C.c_void_p, C.c_int64, C.c_void_p, C.c_uint32, C.POINTER(C.c_int64)]),
    ("fdbcs_sample_attach", C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]),
    ("fdbcs_strerror", C.c_char_p, [C.c_int]),
    ("fdbcs_version", C.c_char_p, []),
    ("fdbcs_comm_unique_id", C.c_int, [C.c_void_p]),
    ("fdbcs_nth_after", C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_uint32, C.c_void_p]),
    ("fdbcs_sharded_create", C.c_int, [C.POINTER(C.c_void_p), C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_int64, C.POINTER(Config), C.c_void_p, C.POINTER(CommOps)]),
    ("fdbcs_sharded_comm_init", C.c_int, [C.c_void_p, C.c_void_p]),
    ("fdbcs_sharded_abort", C.c_int, [C.c_void_p]),
    ("fdbcs_sharded_destroy", None, [C.c_void_p]),
    ("fdbcs_sharded_clear", C.c_int, [C.c_void_p, C.c_int64]),
    ("fdbcs_sharded_batch_begin", C.c_int, [C.c_void_p]),
    ("fdbcs_sharded_batch_add", C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32]),
    ("fdbcs_sharded_batch_skip", C.c_int, [C.c_void_p, C.c_int32]),
    ("fdbcs_sharded_batch_detect", C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]),
    ("fdbcs_sharded_detect_device", C.c_int, [C.c_void_p, C.POINTER(BatchView), C.c_int64, C.c_int64, C.c_void_p]),
    ("fdbcs_sharded_set_protocol", C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    ("fdbcs_sharded_exchange_stats", C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_int]),
    ("fdbcs_sharded_local", C.c_void_p, [C.c_void_p]),
    ("fdbcs_sharded_removal_key_owner", C.c_int32, [C.c_void_p]),
    ("fdbcs_sharded_header_version", C.c_int64, [C.c_void_p]),
]

WL_FUNCS = [
    ("fdbwl_create", C.c_void_p, [C.c_int32, C.c_int32, C.c_int32]),
    ("fdbwl_destroy", None, [C.c_void_p]),
    ("fdbwl_generate", C.c_int, [C.c_void_p, C.c_int64, C.POINTER(BatchView), C.POINTER(C.c_int64),
                                 C.POINTER(C.c_int64)]),
    ("fdbwl_run_prepare", C.c_void_p, [C.c_void_p, C.c_int64, C.c_int32]),
    ("fdbwl_run_prepare_split", C.c_void_p, [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_int32]),
    ("fdbwl_run_key_bytes", C.c_uint64, [C.c_void_p, C.c_int32]),
    ("fdbwl_run_resolver_sharded", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fdbwl_run_destroy", None, [C.c_void_p]),
    ("fdbwl_run_txns", C.c_int32, [C.c_void_p]),
    ("fdbwl_run_resolver", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fdbwl_run_resolver_sampled", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_double, C.c_double,
                                             C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fdbwl_prefill", C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]),
    ("fdbwl_set_successor", None, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("fdbwl_run_adds", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
]

_lib = None
_wl = None


def _bind(lib, funcs):
    for name, res, args in funcs:
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def lib():
    """The HIP product library.  Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m foundationdb_amd.build`")
        # torch's ROCm runtime first: it ships its own libamdhip64 / librccl,
        # whose sonames then satisfy this library's dependencies.  Loaded the
        # other way round, the process holds two HIP runtimes (heap corruption
        # at exit).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        # RTLD_GLOBAL: the workload library's bench drivers call the C ABI through it
        h = _bind(C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL), FDBCS_FUNCS)
        check_single_hip_runtime()
        _lib = h
    return _lib


def hip_runtimes():
    """Distinct HIP runtime images (libamdhip64, by device + inode) mapped into
    this process, as paths."""
    seen = {}
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split(None, 5)
                if len(parts) == 6 and os.path.basename(parts[5].strip()).startswith("libamdhip64"):
                    seen[(parts[3], parts[4])] = parts[5].strip()
    except OSError:
        return []
    return sorted(set(seen.values()))


def check_single_hip_runtime():
    """Raise if more than one HIP runtime is mapped.  That happens when
    libfdbcs.so (which resolves libamdhip64 by soname) is loaded before torch
    and torch then maps its own copy: two runtimes, two heaps, two device
    contexts -- the heap corruption at exit round 2 traced to import order."""
    rt = hip_runtimes()
    if len(rt) > 1:
        raise RuntimeError("two HIP runtimes are mapped into this process (" + ", ".join(rt) + "): load torch "
                           "before libfdbcs.so (foundationdb_amd._abi.lib() does), or run without torch")


def workload_lib():
    global _wl
    if _wl is None:
        lib()  # (its fdbcs_* symbols resolve the workload library's)
        if not os.path.exists(WL_PATH):
            raise RuntimeError(f"{WL_PATH} is missing: build it with `python -m foundationdb_amd.build`")
        _wl = _bind(C.CDLL(WL_PATH), WL_FUNCS)
    return _wl


class FdbcsError(RuntimeError):
    """A nonzero fdbcs status: the reference's ASSERT -> internal_error()."""

    def __init__(self, status, what=""):
        msg = lib().fdbcs_strerror(status).decode()
        super().__init__(f"{what}: fdbcs status {status} ({msg})" if what else f"fdbcs status {status} ({msg})")
        self.status = status


def check(status, what=""):
    if status < 0:
        raise FdbcsError(status, what)
    return status
