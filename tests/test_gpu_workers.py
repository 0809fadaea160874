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


def _kind(n, T, r, request=0, variant=0):
    from ame_amd import _lib
    L = _lib.lib()
    d = _lib.ame_dims(n, r, T, 0, T, variant)
    return int(L.ame_sweep_kind(ctypes.byref(d), request))


def test_kind_selection(gpu_device):
    from ame_amd import _lib
    assert _kind(4096, 32, 32) == 22           # config 5 per-rank shape
    assert _kind(1024, 128, 16) == 3           # config 3: v3
    assert _kind(4096, 40, 32) == 21           # 40 x 8 workgroups do not fit: HBM slice
    assert _kind(4096, 32, 32, _lib.AME_SWEEP_V2_SINGLE) == 21
    assert _kind(1024, 128, 16, _lib.AME_SWEEP_V2_AUTO) == 21    # 128 x 8 > co-resident
    assert _kind(64, 3, 8, _lib.AME_SWEEP_V2_AUTO) == 22
    assert _kind(4096, 40, 32, _lib.AME_SWEEP_V2_WORKERS) == -1  # refused, not re-routed
    assert _kind(4096, 32, 32, _lib.AME_SWEEP_V3) == -1          # d = 66 > 64
    assert _kind(4096, 32, 32, 99) == -1


@pytest.mark.parametrize("n,T,r,method,lr", [
    (24, 3, 32, "good", 0.5), (20, 4, 32, "bad", 1.0), (22, 3, 32, "naive", 0.3),
    (2, 2, 32, "good", 1.0), (5, 3, 32, "good", 0.7), (70, 1, 32, "bad", 0.05),
    (301, 2, 32, "good", 0.5), (130, 3, 24, "naive", 0.5)])
def test_workers_vs_oracle(n, T, r, method, lr, gpu_device):
    assert _kind(n, T, r) == 22
    vi = _check_vs_oracle(n, T, r, method, lr, gpu_device)
    assert vi.engine.sweep_kind == 22


@pytest.mark.parametrize("n,T,r,method,lr", [(64, 3, 8, "good", 0.5), (45, 3, 5, "bad", 1.0)])
def test_workers_small_r_vs_oracle(n, T, r, method, lr, gpu_device):
    """r < 32: lanes >= 2r of a worker wave idle; v2 with workers requested."""
    from ame_amd import _lib
    assert _kind(n, T, r, _lib.AME_SWEEP_V2_AUTO) == 22
    vi = _check_vs_oracle(n, T, r, method, lr, gpu_device, sweep_kernel=_lib.AME_SWEEP_V2_WORKERS)
    assert vi.engine.sweep_kind == 22


@pytest.mark.parametrize("n,T,r,method,lr", [(24, 3, 32, "good", 0.5), (30, 3, 32, "naive", 0.5)])
def test_no_workers_vs_oracle(n, T, r, method, lr, gpu_device):
    """The single-workgroup v2 (kind 20) on a shape that would take workers."""
    from ame_amd import _lib
    assert _kind(n, T, r, _lib.AME_SWEEP_V2_SINGLE) == 20
    vi = _check_vs_oracle(n, T, r, method, lr, gpu_device, sweep_kernel=_lib.AME_SWEEP_V2_SINGLE)
    assert vi.engine.sweep_kind == 20


def test_workers_slice_groups(gpu_device):
    """Slices in consecutive groups (slice_group=2), each launch with its own
    workers: bit-equal to one launch over all slices."""
    from ame_amd import TemporalAMEModel
    outs = []
    for g in (0, 2):
        m = TemporalAMEModel(60, 5, 32, seed=3)
        m.generate_data_fast(seed=4)
        vi = _vi(m, "good", 0.5, gpu_device, slice_group=g)
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
