"""Build the native libraries in-tree (no JIT cache, so they travel to the GPU box).

  foundationdb_amd/libfdbcs.so           product: HIP kernels + C ABI (include/fdbcs.h)
  foundationdb_amd/libfdbcs_workload.so  synthetic batch generators (bench / tests)
  oracle/liboracle_spec.so               CPU restatement (test infrastructure only)

hipcc cross-compiles gfx950 code objects without a GPU, so this runs in the
CPU container.  Each object is rebuilt only when a source or header is newer.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "foundationdb_amd")
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(ROOT, "build", os.environ.get("FDBCS_OBJ_DIR", "obj"))
ARCH = os.environ.get("FDBCS_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["scan.hip", "kernels_batch.hip", "kernels_hist.hip", "engine.hip", "stage.hip", "resolvers.hip",
               "load_metrics.hip"]
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result", "-Wno-unused-value"]
HIP_FLAGS += os.environ.get("FDBCS_EXTRA_FLAGS", "").split()  # experiment variants (scripts/build_variants.sh)
if os.environ.get("FDBCS_PHASES"):  # profiling build: kernels record phase timestamps
    HIP_FLAGS.append("-DFDBCS_PHASES")

# FDBCS_LIB_OUT / FDBCS_OBJ_DIR: build an experiment variant beside the product library
LIB = os.environ.get("FDBCS_LIB_OUT") or os.path.join(PKG, "libfdbcs.so")
WL_LIB = os.path.join(PKG, "libfdbcs_workload.so")
ORACLE_LIB = os.path.join(ROOT, "oracle", "liboracle_spec.so")


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(ROOT, "include", "fdbcs.h"))
    return hs


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
    return p


def build_hip(verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    hdrs = _headers()
    jobs = []
    objs = []
    for src in HIP_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src.replace(".hip", ".o"))
        objs.append(o)
        if _stale(o, [s] + hdrs):
            jobs.append(["hipcc", *HIP_FLAGS, "-c", s, "-o", o])
    workers = min(8, max(1, len(jobs)))
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if _stale(LIB, objs):
        _run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs, "-L/opt/rocm/lib", "-lrccl"],
             verbose)
    return LIB


def build_workload(verbose=False):
    s = os.path.join(CSRC, "workload.cpp")
    deps = [s, os.path.join(CSRC, "workload.h"), os.path.join(ROOT, "include", "fdbcs.h")]
    if _stale(WL_LIB, deps):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", WL_LIB, s, "-ldl"], verbose)
    return WL_LIB


def build_oracle(verbose=False):
    s = os.path.join(ROOT, "oracle", "cpu_spec.cpp")
    if _stale(ORACLE_LIB, [s, os.path.join(ROOT, "include", "fdbcs.h")]):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", ORACLE_LIB, s], verbose)
    return ORACLE_LIB


SHIM = os.path.join(PKG, "shim", "ConflictSetShim.cpp")
SHIM_CHECK = os.path.join(ROOT, "tests", "shim", "shim_smoke")
REF_HEADER_DIR = os.environ.get("FDBCS_REFERENCE", "/root/reference")


def build_shim_check(verbose=False):
    """Compile the ConflictSet.h drop-in TU against the reference's own
    fdbserver/ConflictSet.h (present only in the build container) and link it
    with libfdbcs.so into tests/shim/shim_smoke, which the GPU tests run.
    Skipped (returns None) where the reference tree is absent."""
    hdr = os.path.join(REF_HEADER_DIR, "fdbserver", "ConflictSet.h")
    if not os.path.exists(hdr):
        return None
    main = os.path.join(ROOT, "tests", "shim", "shim_main.cpp")
    stub = os.path.join(ROOT, "tests", "shim", "stub")
    deps = [SHIM, main, os.path.join(stub, "fdbclient", "CommitTransaction.h"), LIB,
            os.path.join(ROOT, "include", "fdbcs.h")]
    if _stale(SHIM_CHECK, deps):
        _run(["g++", "-std=c++17", "-O2", "-Wall", "-pthread", "-iquote", stub, "-iquote", REF_HEADER_DIR, "-I",
              os.path.join(ROOT, "include"), SHIM, main, "-L", PKG, "-lfdbcs",
              "-Wl,-rpath,$ORIGIN/../../foundationdb_amd", "-o", SHIM_CHECK], verbose)
    return SHIM_CHECK


def build_all(verbose=False):
    with ThreadPoolExecutor(3) as ex:
        fs = [ex.submit(build_hip, verbose), ex.submit(build_workload, verbose), ex.submit(build_oracle, verbose)]
        out = [f.result() for f in fs]
    out.append(build_shim_check(verbose))
    return out


if __name__ == "__main__":
    for p in build_all(verbose="-v" in sys.argv):
        print(p)
