"""GPU parity of the pipelined GEMV-worker sweep (kind 23, AME_SWEEP_V2_PIPE;
DESIGN.md §4 K1d), through the C-ABI.

Four worker workgroups per slice (five workgroups per slice instead of kind
22's eight) so that TWO launches are co-resident: the kernel orders itself
slice by slice on the device (per-slice done flags, wait_epoch, the same epoch
window as the v3 sweep), consecutive sweeps overlap and consecutive slice
groups of one sweep overlap.  Checks:

* kind resolution and its co-residency limit;
* the fp64 oracle at small shapes, good / bad / naive, r = 32 and smaller r
  (tolerances of tests/test_gpu_large.py);
* the production schedule (speculative sweeps queued two deep, pipelined, slice
  groups alternating streams) bit for bit the in-order schedule, including
  fits that continue, and slice groups bit for bit one launch;
* config 5's per-rank shape (n=4096, T=32, r=32) in two pipelined groups of 16:
  the second sweep's first 600 nodes of every slice against the fp64 oracle.

Reference: structured_mf.py:211-326, naive_mf.py:207-282.
"""
import ctypes

import numpy as np
import pytest
import torch

from test_gpu_large import _check_vs_oracle, _params, _vi

pytestmark = pytest.mark.gpu

PIPE = 23   # _lib.AME_SWEEP_V2_PIPE


def _kind(n, T, r, request=0, variant=0):
    from ame_amd import _lib
    L = _lib.lib()
    d = _lib.ame_dims(n, r, T, 0, T, variant)
    return int(L.ame_sweep_kind(ctypes.byref(d), request))


def test_pipe_kind_resolution(gpu_device):
    from ame_amd import _lib
    L = _lib.lib()
    assert _lib.AME_SWEEP_V2_PIPE == PIPE
    assert _kind(4096, 32, 32, PIPE) == PIPE
    assert L.ame_sweep_orders_slices(4096, 32, PIPE) == 1
    assert L.ame_sweep_orders_slices(4096, 32, _lib.AME_SWEEP_V2_WORKERS) == 0
    cap = int(L.ame_sweep_max_slices(4096, 32, PIPE))
    assert cap >= 50                            # 5 workgroups per slice, one per CU
    assert _kind(4096, cap, 32, PIPE) == PIPE
    assert _kind(4096, cap + 1, 32, PIPE) == -1   # refused, not re-routed
    assert _kind(5000, 4, 32, PIPE) == -1          # n > 4 x 4 x 256 worker slots


@pytest.mark.parametrize("n,T,r,method,lr", [
    (24, 3, 32, "good", 0.5), (20, 4, 32, "bad", 1.0), (22, 3, 32, "naive", 0.3),
    (2, 2, 32, "good", 1.0), (5, 3, 32, "good", 0.7), (70, 1, 32, "bad", 0.05),
    (301, 4, 32, "good", 0.5), (130, 3, 24, "naive", 0.5), (64, 3, 8, "good", 0.5)])
def test_pipe_vs_oracle(n, T, r, method, lr, gpu_device):
    vi = _check_vs_oracle(n, T, r, method, lr, gpu_device, sweep_kernel=PIPE)
    assert vi.engine.sweep_kind == PIPE and vi.engine.pipelined


def _fit(n, T, r, method, lr, dev, iters, **opts):
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(n, T, r, seed=31)
    m.generate_data_fast(device=dev, seed=32)
    vi = _vi(m, method, lr, dev, sweep_kernel=PIPE, **opts)
    eng = vi.engine
    h = vi.fit(max_iter=iters, tolerance=0.0, verbose=False)
    h2 = vi.fit(max_iter=2, tolerance=0.0, verbose=False)   # a continued fit
    return (eng, vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy(),
            [float(e) for e in h["elbo"] + h2["elbo"]])


@pytest.mark.parametrize("n,T,r,method,group", [
    (200, 12, 32, "good", 0), (150, 10, 32, "bad", 4), (180, 9, 32, "naive", 3),
    (96, 8, 16, "good", 2)])
def test_pipelined_schedule_is_exact(n, T, r, method, group, gpu_device):
    """Speculative, pipelined, slice groups alternating streams (groups of
    `group` slices; 0 = one launch) vs one launch, in order, no speculation."""
    eng, m_p, c_p, e_p = _fit(n, T, r, method, 0.6, gpu_device, 5, slice_group=group)
    assert eng.pipelined and eng.spec_depth >= 2
    assert len(eng.groups) == (1 if group == 0 else -(-T // group))
    eng2, m_s, c_s, e_s = _fit(n, T, r, method, 0.6, gpu_device, 5, speculate=False,
                               pipeline=False)
    assert not eng2.pipelined
    assert np.array_equal(m_p, m_s)
    assert np.array_equal(c_p, c_s)
    assert e_p == e_s


@pytest.mark.timeout(600)
def test_config5_rank_shape_pipelined(gpu_device):
    """BASELINE config 5's per-rank shape on kind 23: two pipelined slice groups
    of 16 (5 x 16 workgroups each, both co-resident).  The production schedule
    (one 3-iteration fit: speculative, pipelined) is bit for bit the in-order
    one (one iteration per fit call), and the in-order run's second sweep --
    the first 600 nodes of all 32 slices, past the 4-node look-behind of the
    workers' partials -- matches the fp64 oracle's replay."""
    import ame_oracle as O
    from ame_amd import TemporalAMEModel
    n, T, r, lr, KF = 4096, 32, 32, 0.01, 600

    def model():
        m = TemporalAMEModel(n, T, r, seed=42)
        m.generate_data_fast(device=gpu_device, seed=42)
        return m

    vi = _vi(model(), "good", lr, gpu_device, sweep_kernel=PIPE)
    assert vi.engine.sweep_kind == PIPE and len(vi.engine.groups) == 2 and vi.engine.pipelined
    vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    prod_m = vi.engine.means_local().cpu().numpy()
    prod_c = vi.engine.covs_local()[:KF].cpu().numpy()
    del vi
    torch.cuda.empty_cache()
    m = model()
    vi = _vi(m, "good", lr, gpu_device, sweep_kernel=PIPE, speculate=False, pipeline=False)
    eng = vi.engine
    assert not eng.pipelined
    vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    x1 = eng.means_local().cpu().numpy().astype(np.float64)
    c1 = eng.covs_local()[:KF].cpu().numpy().astype(np.float64)
    vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    got_m = eng.means_local().cpu().numpy()
    got_c = eng.covs_local()[:KF].cpu().numpy()
    vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    assert np.array_equal(eng.means_local().cpu().numpy(), prod_m)
    assert np.array_equal(eng.covs_local()[:KF].cpu().numpy(), prod_c)
    YK = m.Y[:KF].cpu().numpy()
    del vi, eng
    torch.cuda.empty_cache()
    O.sweep_stats(YK, x1, c1, _params(m), "good", lr, nodes=range(KF))
    err = np.abs(got_m[:KF].astype(np.float64) - x1[:KF]).max()
    cerr = np.abs(got_c.astype(np.float64) - c1).max()
    print(f"config 5 rank shape, kind 23: nodes 0..{KF - 1} vs fp64 oracle: max|dmean| "
          f"{err:.3e} (max|mean| {np.abs(x1[:KF]).max():.3f}), max|dcov| {cerr:.3e}")
    assert err <= 5e-6 * max(1.0, np.abs(x1[:KF]).max()), err
    assert cerr <= 1e-6 * max(1.0, np.abs(c1).max()), cerr
