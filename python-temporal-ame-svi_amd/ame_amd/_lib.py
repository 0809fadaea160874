"""ctypes binding of libame_amd.so (C ABI declared in include/ame_amd.h).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded, :func:`lib` raises ``RuntimeError`` with the reason.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AME_LIB_PATH") or os.path.join(_HERE, "libame_amd.so")

AME_GOOD, AME_BAD, AME_NAIVE = 0, 1, 2
AME_STATUS_SPIN_TIMEOUT = 1
AME_STATUS_HALO_TIMEOUT = 2
AME_STATUS_LDS_TIMEOUT = 4
AME_STATUS_STALE_EPOCH = 8
# the status block (include/ame_amd.h): bits, first-failure record, bookkeeping
AME_STATUS_WORDS = 16
AME_WAIT_SITES = {1: "done flag of slice t (previous sweep)",
                  2: "done flag of slice t+1 (previous sweep)",
                  3: "back channel of the right rank (previous sweep)",
                  4: "hand-off granule of slice t-1",
                  5: "hand-off granule of the left rank's last slice",
                  6: "LDS counter inside the workgroup",
                  7: "GEMV worker: new-mean granule of its slice",
                  8: "slice workgroup: GEMV worker partial"}
AME_PEER_HANDLE_BYTES = 64
# sweep kernel requests / kinds (enum ame_sweep_kind_code)
AME_SWEEP_AUTO, AME_SWEEP_V2_SINGLE, AME_SWEEP_V2_AUTO, AME_SWEEP_V3 = 0, 1, 2, 3
AME_SWEEP_V2_LDS, AME_SWEEP_V2_HBM, AME_SWEEP_V2_WORKERS, AME_SWEEP_V2_PIPE, AME_SWEEP_V2_W6 = 20, 21, 22, 23, 24
AME_SWEEP_FLAG_NEXT_GROUP = 1
AME_SWEEP_FLAG_PREV_GROUP = 2
# ELBO pair kernels (enum ame_pairs_kernel_code)
AME_PAIRS_AUTO, AME_PAIRS_V1, AME_PAIRS_V2 = 0, 1, 2

c_int32 = ctypes.c_int32
c_vp = ctypes.c_void_p


class ame_dims(ctypes.Structure):
    _fields_ = [("n", c_int32), ("r", c_int32), ("T_local", c_int32), ("t_begin", c_int32),
                ("T_total", c_int32), ("variant", c_int32)]


class ame_sweep_args(ctypes.Structure):
    _fields_ = [("Yt", c_vp), ("x_old", c_vp), ("x_new", c_vp), ("next_old", c_vp),
                ("hand", c_vp), ("halo_in", c_vp), ("halo_out", c_vp), ("cov", c_vp),
                ("consts", c_vp), ("rinv", ctypes.c_double * 4), ("lr", ctypes.c_float),
                ("one_minus_lr", ctypes.c_float), ("epoch", ctypes.c_uint32), ("status", c_vp),
                ("work", c_vp), ("cov_new", c_vp), ("done", c_vp),
                ("wait_epoch", ctypes.c_uint32), ("back_out", c_vp), ("back_in", c_vp),
                ("kind", c_int32), ("flags", ctypes.c_uint32), ("work_doubles", ctypes.c_uint64)]


class ame_cov_args(ctypes.Structure):
    _fields_ = [("cov", c_vp), ("consts", c_vp), ("cov_terms", c_vp)]


class ame_elbo_args(ctypes.Structure):
    _fields_ = [("Yt", c_vp), ("x", c_vp), ("prev_final", c_vp), ("cov_terms", c_vp),
                ("consts", c_vp), ("phi", c_vp), ("rinv", ctypes.c_double * 4),
                ("swap_consistent", c_int32), ("work", c_vp), ("out", c_vp),
                ("pairs_kernel", c_int32)]


# every symbol include/ame_amd.h declares (checked by tests/test_capi.py)
EXPORTS = ("ame_pack_y", "ame_pack_y_size", "ame_sweep", "ame_sweep_kind", "ame_sweep_work_size", "ame_sweep_orders_slices", "ame_sweep_max_slices", "ame_sweep_slice_workgroups", "ame_sweep_lds_bytes", "ame_cov",
           "ame_elbo", "ame_elbo_work_size", "ame_elbo_pairs_diag", "ame_host_register", "ame_host_unregister",
           "ame_stream_create_cu_range", "ame_stream_destroy",
           "ame_peer_alloc", "ame_peer_free", "ame_peer_open", "ame_peer_close",
           "ame_peer_probe", "ame_peer_read_u64", "ame_peer_clear",
           "ame_supported_r", "ame_last_error", "ame_version", "ame_align_work_size",
           "ame_align_cross_size", "ame_align_partials_size", "ame_align_cross", "ame_align_apply")

_lock = threading.Lock()
_lib = None


def _declare(L):
    P = ctypes.POINTER
    L.ame_pack_y.argtypes = [c_vp, c_vp, P(ame_dims), c_vp, c_vp]
    L.ame_pack_y_size.argtypes = [P(ame_dims)]
    L.ame_pack_y_size.restype = ctypes.c_longlong
    L.ame_sweep.argtypes = [P(ame_dims), P(ame_sweep_args), c_vp]
    L.ame_sweep_max_slices.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.ame_sweep_lds_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.ame_sweep_lds_bytes.restype = ctypes.c_longlong
    L.ame_cov.argtypes = [P(ame_dims), P(ame_cov_args), c_vp]
    L.ame_elbo.argtypes = [P(ame_dims), P(ame_elbo_args), c_vp]
    L.ame_elbo_pairs_diag.argtypes = [P(ame_dims), P(ame_elbo_args), c_vp]
    L.ame_elbo_pairs_diag.restype = ctypes.c_int
    L.ame_debug_gw_tag.argtypes = [ctypes.c_uint, ctypes.c_int]
    L.ame_debug_gw_tag.restype = ctypes.c_uint
    L.ame_elbo_work_size.argtypes = [P(ame_dims)]
    L.ame_elbo_work_size.restype = ctypes.c_longlong
    L.ame_debug_selftest.argtypes = [c_vp, c_vp]
    L.ame_debug_selftest.restype = ctypes.c_int
    if hasattr(L, "ame_debug_occupy"):   # diagnostic; absent from older A/B builds
        L.ame_debug_occupy.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint, c_vp, c_vp]
        L.ame_debug_occupy.restype = ctypes.c_int
    if hasattr(L, "ame_sweep_slice_workgroups"):   # absent from older A/B builds only
        L.ame_sweep_slice_workgroups.argtypes = [ctypes.c_int]
        L.ame_sweep_slice_workgroups.restype = ctypes.c_int
    L.ame_sweep_orders_slices.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.ame_sweep_orders_slices.restype = ctypes.c_int
    L.ame_sweep_kind.argtypes = [P(ame_dims), ctypes.c_int]
    L.ame_sweep_kind.restype = ctypes.c_int
    L.ame_sweep_work_size.argtypes = [P(ame_dims), ctypes.c_int]
    L.ame_sweep_work_size.restype = ctypes.c_longlong
    L.ame_supported_r.argtypes = [P(ctypes.c_int), ctypes.c_int]
    L.ame_stream_create_cu_range.argtypes = [ctypes.c_int, ctypes.c_int, P(c_vp)]
    L.ame_stream_destroy.argtypes = [c_vp]
    L.ame_host_register.argtypes = [c_vp, ctypes.c_ulonglong, P(c_vp)]
    L.ame_host_unregister.argtypes = [c_vp]
    L.ame_peer_alloc.argtypes = [ctypes.c_ulonglong, P(c_vp), c_vp]
    L.ame_peer_free.argtypes = [c_vp]
    L.ame_peer_open.argtypes = [c_vp, P(c_vp)]
    L.ame_peer_close.argtypes = [c_vp]
    L.ame_peer_probe.argtypes = [c_vp, ctypes.c_ulonglong]
    L.ame_peer_read_u64.argtypes = [c_vp, P(ctypes.c_ulonglong)]
    L.ame_peer_clear.argtypes = [c_vp, ctypes.c_ulonglong]
    ci = ctypes.c_int
    for name in ("ame_align_work_size", "ame_align_cross_size"):
        getattr(L, name).restype = ctypes.c_longlong
    L.ame_align_work_size.argtypes = [ci, ci, ci]
    L.ame_align_cross_size.argtypes = [ci, ci, ci, ci]
    L.ame_align_partials_size.argtypes = [ci, ci]
    L.ame_align_partials_size.restype = ctypes.c_longlong
    L.ame_align_cross.argtypes = [c_vp, c_vp, ci, ci, ci, ci, c_vp, c_vp, c_vp]
    L.ame_align_cross.restype = ci
    L.ame_align_apply.argtypes = [c_vp, c_vp, ci, ci, ci, ci, c_vp, c_vp, c_vp, c_vp]
    L.ame_align_apply.restype = ci
    L.ame_last_error.restype = ctypes.c_char_p
    L.ame_version.restype = ctypes.c_char_p
    for name in ("ame_pack_y", "ame_sweep", "ame_cov", "ame_elbo", "ame_sweep_max_slices",
                 "ame_supported_r", "ame_host_register", "ame_host_unregister", "ame_peer_alloc",
                 "ame_peer_free", "ame_peer_open", "ame_peer_close", "ame_peer_probe",
                 "ame_peer_read_u64", "ame_peer_clear"):
        getattr(L, name).restype = ctypes.c_int
    return L


def lib():
    """Load libame_amd.so (built by ame_amd.build / __graft_entry__.build())."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"ame_amd: HIP library not found at {LIB_PATH}; run "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
            try:
                _lib = _declare(ctypes.CDLL(LIB_PATH))
            except OSError as e:  # pragma: no cover - depends on the box
                raise RuntimeError(f"ame_amd: cannot load {LIB_PATH}: {e}") from e
        return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().ame_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def build_hash():
    """The source hash the loaded library was built from (ame_version "src=")."""
    v = lib().ame_version().decode(errors="replace")
    return v.split("src=", 1)[1] if "src=" in v else None


def provenance():
    """{lib, tree, match}: the loaded library's source hash against the hash of
    the sources beside it (ame_amd/build.py), so a stale library is visible."""
    from .build import source_hash
    got = build_hash()
    try:
        tree = source_hash()
    except OSError:   # pragma: no cover - sources not shipped
        tree = None
    return {"lib_src": got, "tree_src": tree, "match": got is not None and got == tree,
            "path": LIB_PATH}


def supported_r():
    L = lib()
    buf = (ctypes.c_int * 64)()
    k = L.ame_supported_r(buf, 64)
    return tuple(buf[i] for i in range(min(k, 64)))
