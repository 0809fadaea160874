"""The C-ABI library loads and exports every symbol include/ame_amd.h declares.

No compute calls here (no GPU in the build container): only the host-side
entry points that never touch the device, and argument validation, which
returns before any HIP call.
"""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _lib():
    from ame_amd import _lib as L
    if not os.path.exists(L.LIB_PATH):
        from ame_amd.build import build
        build(verbose=False)
    return L


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "ame_amd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ame_[a-z_0-9]+)\s*\(", txt)))


def test_header_symbols_exported():
    L = _lib()
    lib = L.lib()
    syms = _header_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/ame_amd.h but not exported"
    assert set(syms) == set(L.EXPORTS)


def test_host_only_entry_points():
    L = _lib()
    lib = L.lib()
    assert b"gfx950" in lib.ame_version()
    rs = L.supported_r()
    # every latent dim 1..32 is compiled (the reference takes any r,
    # temporal_ame.py:114-120); the split build routes each r to its part
    assert list(rs) == list(range(1, 33))
    for r in (9, 10, 17, 31, 32):
        assert lib.ame_sweep_lds_bytes(64, r, L.AME_SWEEP_V2_LDS) > 0
    # LDS budget of the v2 sweep's per-slice state: config 3 (n=1024, r=16) fits one CU
    assert 0 < lib.ame_sweep_lds_bytes(1024, 16, L.AME_SWEEP_V2_LDS) <= 160 * 1024
    assert lib.ame_sweep_lds_bytes(1024, 999, L.AME_SWEEP_V2_LDS) == 0
    assert lib.ame_sweep_lds_bytes(1024, 16, 7) == 0              # not a concrete kind
    d = L.ame_dims(1024, 16, 128, 0, 128, L.AME_GOOD)
    assert lib.ame_elbo_work_size(ctypes.byref(d)) > 0
    # scratch of each concrete kind (host arithmetic, no device query)
    assert lib.ame_sweep_work_size(ctypes.byref(d), L.AME_SWEEP_V2_LDS) == 0
    assert lib.ame_sweep_work_size(ctypes.byref(d), L.AME_SWEEP_V2_HBM) == 128 * 1024 * 32 // 2
    assert lib.ame_sweep_work_size(ctypes.byref(d), L.AME_SWEEP_V2_WORKERS) == 128 * 7 * 8 * 34 + 128 * 1024 * 4 * 34
    assert lib.ame_sweep_work_size(ctypes.byref(d), 2) == -1     # a request, not a kind
    # workgroups per slice (the engine's elbo_cus sizing reads these)
    assert [lib.ame_sweep_slice_workgroups(k) for k in (3, 20, 21, 22, 23, 24)] == [1, 1, 1, 8, 5, 7]
    assert lib.ame_sweep_slice_workgroups(L.AME_SWEEP_AUTO) == -1


def test_worker_partial_tag_never_zero():
    """GEMV-worker partial tags (ame_common.h ame_gw_tag): a slot the launch
    zeroed must never carry a valid tag, including epoch 65536 (whose low 16
    bits are 0) for node 0."""
    lib = _lib().lib()
    for epoch in (1, 2, 32768, 65535, 65536, 65537, 2 ** 31, 2 ** 32 - 1):
        for m in (0, 1, 7, 4095, 65535):
            tag = lib.ame_debug_gw_tag(epoch, m)
            assert tag != 0 and (tag & 0xFFFF) == m
    # consecutive epochs (one launch each) and ring neighbours m, m + 8 differ
    assert lib.ame_debug_gw_tag(65536, 0) != lib.ame_debug_gw_tag(65537, 0)
    assert lib.ame_debug_gw_tag(5, 0) != lib.ame_debug_gw_tag(5, 8)


def test_argument_validation_fails_loudly():
    L = _lib()
    lib = L.lib()
    d = L.ame_dims(16, 2, 4, 0, 4, L.AME_GOOD)
    a = L.ame_sweep_args()
    rc = lib.ame_sweep(ctypes.byref(d), ctypes.byref(a), None)
    assert rc != 0 and b"NULL" in lib.ame_last_error()
    bad = L.ame_dims(16, 999, 4, 0, 4, L.AME_GOOD)
    assert lib.ame_sweep(ctypes.byref(bad), ctypes.byref(a), None) != 0
    assert b"latent_dim" in lib.ame_last_error()
    rng = L.ame_dims(16, 2, 4, 2, 4, L.AME_GOOD)   # slices [2, 6) outside T=4
    assert lib.ame_cov(ctypes.byref(rng), ctypes.byref(L.ame_cov_args()), None) != 0
    with pytest.raises(RuntimeError):
        L.check(-1, "ame_sweep")


def test_no_cpu_fallback():
    """The product path refuses to run without a GPU instead of falling back."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    m = TemporalAMEModel(6, 3, 2, seed=1)
    m.generate_data()
    vi = TemporalAMEStructuredMFVI(m)
    with pytest.raises(RuntimeError, match="no GPU"):
        vi.fit(max_iter=1, verbose=False)
