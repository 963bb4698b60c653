"""ctypes binding of ``libsmx.so`` (the C ABI declared in ``include/smx.h``).

The library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()`` runs it).  There
is no fallback of any kind: if the library is missing or fails to load, importing the engine
raises.  The host engine (``smx_host_*``, ``host.py``) is part of the same library and is chosen
only where no HIP device exists (or on request); a HIP device always gets the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SMX_LIB names another build of the same library in this directory (tools: "libsmx_diag.so",
# the sweep path counters of `make -C csrc diag`); the product loads libsmx.so
LIB_PATH = os.path.join(HERE, os.path.basename(os.environ.get("SMX_LIB", "libsmx.so")))

# outcome codes, include/smx.h
PIVOT, OPTIMUM, INCORRECT, NOT_CONVERGE, FSHORT, IDLE = 0, 1, 2, 3, 4, 5
NONE = 0x7F7F7F7F
SHARD_HDR = 8
CTL_BYTES = 128
PART_BYTES = 32

# numpy view of struct smx_ctl (include/smx.h)
CTL_DTYPE = np.dtype([
    ("negb", "<i4", (2,)), ("negf", "<i4", (2,)), ("term", "<i4"), ("sel_status", "<i4"),
    ("sel_r", "<i4"), ("sel_c", "<i4"), ("sel_e", "<f8"), ("npivots", "<i8"),
    ("sel_owner", "<i4"), ("nla", "<i4"), ("shard_off", "<i8"), ("xpos", "<i4", (2, 2)),
    ("npiv", "<i8", (2,)), ("dec", "<i4", (2, 4)),
])
ABSENT = -0x80000000
assert CTL_DTYPE.itemsize == CTL_BYTES


class Shape(ctypes.Structure):
    """struct smx_shape (include/smx.h)."""
    _fields_ = [("ld", ctypes.c_int64), ("rows", ctypes.c_int32), ("n", ctypes.c_int32),
                ("m", ctypes.c_int32), ("flen", ctypes.c_int32), ("row0", ctypes.c_int32),
                ("nparts", ctypes.c_int32)]


class Rank(ctypes.Structure):
    """struct smx_rank (include/smx.h): one row block of a single-process multi-device table."""
    _fields_ = [("device", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("stream", ctypes.c_void_p), ("buf0", ctypes.c_void_p),
                ("buf1", ctypes.c_void_p), ("ctl", ctypes.c_void_p), ("blk", ctypes.c_void_p),
                ("blk_bytes", ctypes.c_int64), ("send", ctypes.c_void_p),
                ("recv", ctypes.c_void_p), ("log", ctypes.c_void_p), ("xhist", ctypes.c_void_p),
                ("log_cap", ctypes.c_int64), ("comm", ctypes.c_void_p), ("shape", Shape)]


XCHG_RCCL, XCHG_COPY = 0, 1
ERR_COMMS_ABORTED = -2000   # smx_mshard_run: a rank failed, every communicator was aborted

_lib = None

CSRC = os.path.join(os.path.dirname(HERE), "csrc")
INCLUDE_H = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "smx.h")


def source_stamp() -> str | None:
    """The stamp csrc/Makefile compiles into the library (SRC_HASH): the first 16 hex digits of
    the SHA-256 of include/smx.h, csrc/*.hpp in name order and csrc/smx_kernels.hip, concatenated;
    None where the sources are not next to the package."""
    import glob
    import hashlib
    kern = os.path.join(CSRC, "smx_kernels.hip")
    if not (os.path.exists(kern) and os.path.exists(INCLUDE_H)):
        return None
    files = [INCLUDE_H] + sorted(glob.glob(os.path.join(CSRC, "*.hpp"))) + [kern]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def library_stamp(L) -> str | None:
    buf = ctypes.create_string_buffer(256)
    L.smx_version(buf, 256)
    v = buf.value.decode()
    return v.split("src=", 1)[1].split()[0] if "src=" in v else None


def check_stamp(L, path: str) -> None:
    """Refuse a libsmx build whose source stamp differs from the sources in this tree (the
    product and the diagnostic build share the stamp; other SMX_LIB builds -- A/B variants built
    from edited sources on purpose -- are not checked)."""
    if os.path.basename(path) not in ("libsmx.so", "libsmx_diag.so"):
        return
    want = source_stamp()
    if want is None:
        return
    got = library_stamp(L)
    if got != want:
        raise OSError(f"{path} is stale: built from sources stamped {got!r}, the tree's sources "
                      f"are {want!r}; rebuild it (`make -C simplex-method-solver_amd/csrc` or "
                      "__graft_entry__.build())")


EXPORTS = (
    "smx_version", "smx_nparts_for", "smx_tune_set", "smx_tune_get", "smx_tune_fused",
    "smx_set_xpos", "smx_reset", "smx_select", "smx_finalize", "smx_update",
    "smx_run", "smx_run_timed", "smx_graph_create", "smx_graph_launch", "smx_graph_destroy", "smx_update_forced",
    "smx_batch_solve", "smx_comm_unique_id", "smx_comm_init", "smx_comm_destroy",
    "smx_shard_run", "smx_shard_run_timed", "smx_shard_pack", "smx_shard_merge", "smx_shard_update", "smx_shard_begin",
    "smx_shard_finish", "smx_shard_fused_prime", "smx_shard_fused_begin",
    "smx_shard_fused_finish", "smx_fused_publish", "smx_shard_ahead", "smx_shard_sweep",
    "smx_copy_probe", "smx_shard_folds_pack", "smx_tune_fold",
    "smx_tune_resident", "smx_tune_resident_overlap", "smx_tune_resident_timeout", "smx_resident_trace", "smx_resident_bytes",
    "smx_resident_run", "smx_fastdiv_check", "smx_fastdiv_check_bounded",
    "smx_tune_block", "smx_tune_block_form", "smx_tune_block_planner", "smx_block_bytes", "smx_block_run", "smx_block_run_timed",
    "smx_block_timed_read",
    "smx_block_graph_create",
    "smx_bshard_bytes", "smx_bshard_run", "smx_bshard_run_timed", "smx_bshard_graph_create",
    "smx_bshard_prime",
    "smx_bshard_pack", "smx_bshard_step", "smx_bshard_sweep", "smx_bshard_publish",
    "smx_bshard_pick", "smx_bshard_step_light", "smx_tune_shard_xchg",
    "smx_host_select", "smx_host_pivot", "smx_host_run", "smx_timer_reserve",
    "smx_mshard_comms", "smx_mshard_run", "smx_int_first_fix", "smx_host_int_first_fix",
    "smx_diag_path_counts", "smx_comm_info", "smx_mshard_graph_create", "smx_mshard_last_error",
)


def load():
    """Load libsmx.so once; raises OSError if it is missing (build it with csrc/Makefile)."""
    global _lib
    if _lib is not None:
        return _lib
    # torch first: libsmx.so and torch's bundled runtime share the SONAME libamdhip64.so.7, and
    # the engine must run on the runtime torch already initialised (one HIP runtime per process)
    import torch  # noqa: F401
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not built: run `make -C simplex-method-solver_amd/csrc` "
                      "(or __graft_entry__.build()); the engine has no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    L.smx_version.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.smx_version.restype = ctypes.c_int
    check_stamp(L, LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sp = ctypes.POINTER(Shape)
    sig = {
        "smx_version": ([ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
        "smx_nparts_for": ([i32, i32], ctypes.c_int),
        "smx_tune_set": ([i32, i32], ctypes.c_int),
        "smx_tune_fused": ([i32], ctypes.c_int),
        "smx_tune_get": ([ctypes.POINTER(i32)] * 6, ctypes.c_int),
        "smx_reset": ([vp, sp, i32, i32, vp, vp], ctypes.c_int),
        "smx_select": ([vp, sp, i32, vp, vp, vp], ctypes.c_int),
        "smx_finalize": ([vp, sp, i32, vp, vp, vp], ctypes.c_int),
        "smx_update": ([vp, vp, sp, i32, vp, vp, vp, vp, i64, vp], ctypes.c_int),
        "smx_set_xpos": ([vp, i32, i32, i32, vp], ctypes.c_int),
        "smx_run": ([vp, vp, sp, i32, i32, vp, vp, vp, vp, i64, vp], ctypes.c_int),
        "smx_run_timed": ([vp, vp, sp, i32, i32, vp, vp, vp, vp, i64, vp,
                           ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)],
                          ctypes.c_int),
        "smx_graph_create": ([vp, vp, sp, i32, i32, vp, vp, vp, vp, i64, vp,
                              ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
        "smx_graph_launch": ([vp, vp], ctypes.c_int),
        "smx_graph_destroy": ([vp], ctypes.c_int),
        "smx_update_forced": ([vp, vp, sp, i32, i32, vp], ctypes.c_int),
        "smx_shard_pack": ([vp, sp, i32, vp, vp, vp, vp], ctypes.c_int),
        "smx_shard_merge": ([vp, i32, sp, i32, vp, vp, i64, vp], ctypes.c_int),
        "smx_shard_update": ([vp, vp, vp, i32, sp, i32, vp, vp, i64, vp], ctypes.c_int),
        "smx_comm_unique_id": ([vp], ctypes.c_int),
        "smx_comm_init": ([ctypes.POINTER(ctypes.c_void_p), i32, vp, i32], ctypes.c_int),
        "smx_comm_destroy": ([vp], ctypes.c_int),
        "smx_shard_run": ([vp, vp, sp, i32, i32, vp, vp, vp, vp, i32, vp, vp, i64, vp],
                          ctypes.c_int),
        "smx_shard_run_timed": ([vp, vp, sp, i32, i32, vp, vp, vp, vp, i32, vp, vp, i64, vp,
                                 ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)],
                                ctypes.c_int),
        "smx_batch_solve": ([vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp],
                            ctypes.c_int),
        "smx_shard_begin": ([vp, sp, i32, vp, vp, vp, vp], ctypes.c_int),
        "smx_shard_finish": ([vp, vp, vp, i32, sp, i32, vp, vp, i64, vp, vp, vp], ctypes.c_int),
        "smx_shard_fused_prime": ([vp, sp, i32, vp, vp, vp], ctypes.c_int),
        "smx_shard_fused_begin": ([vp, sp, i32, vp, vp, vp, vp], ctypes.c_int),
        "smx_shard_fused_finish": ([vp, vp, vp, i32, sp, i32, vp, vp, vp, vp, i64, vp, vp, vp],
                                   ctypes.c_int),
        "smx_fused_publish": ([sp, i32, vp, vp, vp], ctypes.c_int),
        "smx_shard_ahead": ([vp, sp, i32, vp, i32, vp, vp, vp, vp], ctypes.c_int),
        "smx_shard_sweep": ([vp, vp, vp, i32, sp, i32, vp, vp, i64, vp], ctypes.c_int),
        "smx_copy_probe": ([vp, vp, i64, i32, vp], ctypes.c_int),
        "smx_shard_folds_pack": ([sp], ctypes.c_int),
        "smx_tune_fold": ([i64], ctypes.c_int64),
        "smx_tune_resident": ([i32], ctypes.c_int),
        "smx_tune_resident_overlap": ([i32], ctypes.c_int),
        "smx_tune_resident_timeout": ([i64], ctypes.c_int64),
        "smx_resident_bytes": ([sp, ctypes.POINTER(i32)], ctypes.c_int64),
        "smx_resident_trace": ([vp, i32], ctypes.c_int),
        "smx_resident_run": ([vp, vp, sp, i32, i32, vp, vp, i64, i32, vp, vp, i64, vp],
                             ctypes.c_int),
        "smx_fastdiv_check": ([vp, vp, i64, vp, vp], ctypes.c_int),
        "smx_fastdiv_check_bounded": ([vp, vp, i64, vp, vp], ctypes.c_int),
        "smx_diag_path_counts": ([ctypes.POINTER(i64), i32, i32], ctypes.c_int),
        "smx_comm_info": ([vp] + [ctypes.POINTER(i32)] * 3, ctypes.c_int),
        "smx_mshard_graph_create": ([ctypes.POINTER(Rank), i32, i32, i32, i32,
                                     ctypes.POINTER(vp)], ctypes.c_int),
        "smx_tune_block": ([i32], ctypes.c_int),
        "smx_tune_block_form": ([i32], ctypes.c_int),
        "smx_tune_block_planner": ([i32, i32], ctypes.c_int),
        "smx_block_bytes": ([sp, ctypes.POINTER(i32)], ctypes.c_int64),
        "smx_block_run": ([vp, vp, sp, i32, i32, i32, vp, vp, i64, vp, vp, i64, vp],
                          ctypes.c_int),
        "smx_block_run_timed": ([vp, vp, sp, i32, i32, i32, vp, vp, i64, vp, vp, i64, vp,
                                 ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)],
                                ctypes.c_int),
        "smx_block_timed_read": ([i32, ctypes.POINTER(ctypes.c_float),
                                  ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
        "smx_block_graph_create": ([vp, vp, sp, i32, i32, i32, vp, vp, i64, vp, vp, i64, vp,
                                    ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
        "smx_bshard_bytes": ([sp], ctypes.c_int64),
        "smx_bshard_run": ([vp, vp, sp, i32, i32, i32, vp, vp, i64, vp, vp, i32, vp, vp, vp,
                            i64, vp], ctypes.c_int),
        "smx_bshard_run_timed": ([vp, vp, sp, i32, i32, i32, vp, vp, i64, vp, vp, i32, vp, vp,
                                  vp, i64, vp, ctypes.POINTER(ctypes.c_float),
                                  ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
        "smx_bshard_graph_create": ([vp, vp, sp, i32, i32, i32, vp, vp, i64, vp, vp, i32, vp,
                                     vp, vp, i64, vp, ctypes.POINTER(ctypes.c_void_p)],
                                    ctypes.c_int),
        "smx_bshard_prime": ([vp, sp, i32, vp, vp, i64, vp], ctypes.c_int),
        "smx_bshard_pack": ([vp, sp, i32, i32, i32, vp, vp, i64, vp, vp], ctypes.c_int),
        "smx_bshard_step": ([vp, sp, i32, i32, i32, i32, vp, i32, vp, vp, i64, vp, vp, i64,
                             vp],
                            ctypes.c_int),
        "smx_bshard_sweep": ([vp, vp, sp, i32, vp, i64, vp], ctypes.c_int),
        "smx_bshard_pick": ([vp, sp, i32, i32, vp, vp, vp], ctypes.c_int),
        "smx_bshard_step_light": ([vp, sp, i32, i32, i32, i32, vp, vp, i32, vp, vp, i64, vp, vp,
                                   i64, vp], ctypes.c_int),
        "smx_tune_shard_xchg": ([i32], ctypes.c_int),
        "smx_bshard_publish": ([sp, i32, i32, vp, vp, i64, vp], ctypes.c_int),
        "smx_host_select": ([vp, sp, vp], ctypes.c_int),
        "smx_host_pivot": ([vp, vp, sp, i32, i32], ctypes.c_int),
        "smx_host_run": ([vp, vp, sp, i32, i64, vp, vp], ctypes.c_int64),
        "smx_timer_reserve": ([i32], ctypes.c_int),
        "smx_mshard_comms": ([ctypes.POINTER(ctypes.c_void_p), i32, ctypes.POINTER(i32)],
                             ctypes.c_int),
        "smx_mshard_run": ([ctypes.POINTER(Rank), i32, i32, i32, i32, i32], ctypes.c_int),
        "smx_mshard_last_error": ([ctypes.POINTER(i32)], ctypes.c_int),
        "smx_int_first_fix": ([vp, vp, i64, i32, i32, i32, i32, vp, vp, i64, vp, vp],
                              ctypes.c_int),
        "smx_host_int_first_fix": ([vp, vp, i64, i32, i32, i32, i32, vp, vp, i64, vp],
                                   ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def version() -> str:
    buf = ctypes.create_string_buffer(256)
    load().smx_version(buf, 256)
    return buf.value.decode()


def resident_plan(shape) -> tuple[int, tuple[int, int, int, int]] | None:
    """(exchange bytes, (workgroups, rows per workgroup, elements per thread, LDS bytes)) of the
    on-chip resident pivot loop for ``shape`` = [ld, rows, n, m, flen, row0, nparts], or None
    when the tableau is not eligible (sharded, or its rows do not fit in LDS)."""
    sh = Shape(*(int(x) for x in shape))
    plan = (ctypes.c_int32 * 4)()
    nbytes = load().smx_resident_bytes(ctypes.byref(sh), plan)
    if nbytes <= 0:
        return None
    return int(nbytes), tuple(int(x) for x in plan)


def tune_resident_overlap(on: int = -1) -> int:
    """smx_tune_resident_overlap: 2 automatic (overlapped from 768 columns, the default), 1 the
    overlapped resident loop, 0 the round-3 loop, -1 query only; returns the previous setting."""
    return int(load().smx_tune_resident_overlap(on))


def tune_resident(workgroups: int = -2) -> int:
    """smx_tune_resident: -1 never, 0 automatic, > 0 that many workgroups, -2 query only;
    returns the previous setting."""
    return int(load().smx_tune_resident(workgroups))


def block_plan(shape, pivots: int = 0) -> tuple[int, int] | None:
    """(scratch bytes, pivots per sweep) of the block-pivot chain for ``shape``: with
    ``pivots`` = 0 under the library's policy (smx_tune_block; None when chains of this shape do
    not use blocks), else for that many pivots per sweep (None when not eligible)."""
    sh = Shape(*(int(x) for x in shape))
    piv = ctypes.c_int32(int(pivots))
    nbytes = load().smx_block_bytes(ctypes.byref(sh), ctypes.byref(piv))
    if nbytes <= 0:
        return None
    return int(nbytes), int(piv.value)


def tune_block(pivots: int = -1) -> int:
    """smx_tune_block: 0 automatic, 1 never, 2..24 pivots per sweep, -1 query only; returns the
    previous setting."""
    return int(load().smx_tune_block(pivots))


def tune_block_planner(planner: int = -1, nwin: int = -1) -> int:
    """smx_tune_block_planner: 0 the window planner (the default: one persistent launch per block
    where eligible, else one launch per pivot), 2 the window planner's launch form, 1 the
    register-form chains, -1 query only; ``nwin`` window slots 2..64 (0: 64, -1: keep).  Returns
    the previous planner."""
    return int(load().smx_tune_block_planner(planner, nwin))


def tune_block_form(form: int = -1) -> int:
    """smx_tune_block_form: 0 automatic, 4 pivot-row slices in registers, 5 in LDS, 6 in LDS by
    work items (rows in segments, each at another column chunk); any other
    value only queries; returns the previous setting."""
    return int(load().smx_tune_block_form(form))


def tune_shard_xchg(mode: int = -2) -> int:
    """smx_tune_shard_xchg: -1 automatic (light from 4 ranks on), 0 full send slots, 1 light
    (header all-gather + one max all-reduce of the pivot row), -2 query only; returns the previous
    setting."""
    return int(load().smx_tune_shard_xchg(mode))


BLOCK_MAX = 24   # pivots per sweep at most (kBlkMax)


RESIDENT_TIMEOUT = 1   # smx_ctl.dec[0][0] after a resident hand-off timed out
RESIDENT_EPOCHS = 4095   # tags of one exchange buffer cycle through epochs 1..4095


def fused_enabled() -> bool:
    """True when chains run one fused kernel per pivot (smx_tune_fused; the default)."""
    return bool(load().smx_tune_fused(-1))


NCCL_RESULTS = {1: "ncclUnhandledCudaError", 2: "ncclSystemError", 3: "ncclInternalError",
                4: "ncclInvalidArgument", 5: "ncclInvalidUsage (e.g. two ranks on one GPU)",
                6: "ncclRemoteError", 7: "ncclInProgress"}


def check(err: int, what: str) -> None:
    """Raise on a libsmx error: hipError_t codes, or -1000 - ncclResult_t for RCCL failures."""
    if err == 0:
        return
    if err == ERR_COMMS_ABORTED:
        rank = ctypes.c_int32(-1)
        cause = int(load().smx_mshard_last_error(ctypes.byref(rank)))
        why = ""
        if cause:
            why = (f" (rank {rank.value}: RCCL {NCCL_RESULTS.get(-1000 - cause, -1000 - cause)})"
                   if cause <= -1000 else f" (rank {rank.value}: hipError {cause})")
        raise RuntimeError(f"{what} failed: a rank could not enqueue its chain{why}; every RCCL "
                           "communicator was aborted")
    if err <= -1000:
        code = -1000 - err
        raise RuntimeError(f"{what} failed: RCCL {NCCL_RESULTS.get(code, code)}")
    raise RuntimeError(f"{what} failed with hipError {err}")
