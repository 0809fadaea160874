"""GPU parity of the v2 sweep with GEMV worker workgroups (kind 22; DESIGN.md
§K1c), through the C-ABI.  Seven workgroups per slice hold node ranges of the
slice's (U,V) block and publish per-node partial h_obs sums; the slice's
workgroup adds them in a fixed order plus the two newest nodes.  The h_obs sum
order differs from the single-workgroup v2 (kinds 20 / 21), so the check is
against the fp64 oracle (tolerances as tests/test_gpu_large.py) and run-to-run
bit equality, not against the other kinds.

Reference: structured_mf.py:289-326 (observation term), naive_mf.py:207-282.
"""
import ctypes

import numpy as np
import pytest

from test_gpu_large import _check_vs_oracle, _vi

pytestmark = pytest.mark.gpu


def _kind(n, T, r, variant=0):
    from ame_amd import _lib
    L = _lib.lib()
    d = _lib.ame_dims(n, r, T, 0, T, variant)
    return int(L.ame_sweep_kind(ctypes.byref(d)))


def test_kind_selection(gpu_device, monkeypatch):
    assert _kind(4096, 32, 32) == 22           # config 5 per-rank shape
    assert _kind(1024, 128, 16) == 3           # config 3: v3
    assert _kind(4096, 40, 32) == 21           # 40 x 8 workgroups do not fit: HBM slice
    monkeypatch.setenv("AME_SWEEP_NOWORKERS", "1")
    assert _kind(4096, 32, 32) == 21


@pytest.mark.parametrize("n,T,r,method,lr", [
    (24, 3, 32, "good", 0.5), (20, 4, 32, "bad", 1.0), (22, 3, 32, "naive", 0.3),
    (2, 2, 32, "good", 1.0), (5, 3, 32, "good", 0.7), (70, 1, 32, "bad", 0.05),
    (301, 2, 32, "good", 0.5), (130, 3, 24, "naive", 0.5)])
def test_workers_vs_oracle(n, T, r, method, lr, gpu_device):
    assert _kind(n, T, r) == 22
    vi = _check_vs_oracle(n, T, r, method, lr, gpu_device)
    assert vi.engine.sweep_kind == 22


@pytest.mark.parametrize("n,T,r,method,lr", [(64, 3, 8, "good", 0.5), (45, 3, 5, "bad", 1.0)])
def test_workers_small_r_vs_oracle(n, T, r, method, lr, gpu_device, monkeypatch):
    """r < 32: lanes >= 2r of a worker wave idle; v2 forced (AME_SWEEP_V2=1)."""
    monkeypatch.setenv("AME_SWEEP_V2", "1")
    assert _kind(n, T, r) == 22
    _check_vs_oracle(n, T, r, method, lr, gpu_device)


@pytest.mark.parametrize("n,T,r,method,lr", [(24, 3, 32, "good", 0.5), (30, 3, 32, "naive", 0.5)])
def test_no_workers_vs_oracle(n, T, r, method, lr, gpu_device, monkeypatch):
    """AME_SWEEP_NOWORKERS=1 keeps the single-workgroup v2 (kind 20)."""
    monkeypatch.setenv("AME_SWEEP_NOWORKERS", "1")
    assert _kind(n, T, r) == 20
    _check_vs_oracle(n, T, r, method, lr, gpu_device)


def test_workers_slice_groups(gpu_device, monkeypatch):
    """Slices in consecutive groups (AME_SLICE_GROUP=2), each launch with its own
    workers: bit-equal to one launch over all slices."""
    from ame_amd import TemporalAMEModel
    outs = []
    for g in ("0", "2"):
        monkeypatch.setenv("AME_SLICE_GROUP", g)
        m = TemporalAMEModel(60, 5, 32, seed=3)
        m.generate_data_fast(seed=4)
        vi = _vi(m, "good", 0.5, gpu_device)
        assert vi.engine.sweep_kind == 22
        vi.fit(max_iter=2, tolerance=0.0, verbose=False)
        outs.append((vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])


def test_config5_shape_deterministic(gpu_device):
    """n = 4096, r = 32 on 4 slices: two fits from one seed are bit-equal (the
    worker partials are summed in a fixed order, independent of timing)."""
    from ame_amd import TemporalAMEModel
    outs = []
    for _ in range(2):
        m = TemporalAMEModel(4096, 4, 32, seed=5)
        m.generate_data_fast(seed=6)
        vi = _vi(m, "good", 0.5, gpu_device)
        assert vi.engine.sweep_kind == 22
        vi.fit(max_iter=1, tolerance=0.0, verbose=False)
        outs.append(vi.X_mean.numpy().copy())
    assert np.array_equal(outs[0], outs[1])
