"""GPU parity of the six-worker sweep (kind 24, AME_SWEEP_V2_W6) and of the
ELBO-beside-the-sweep schedule (engine option elbo_cus: CU-masked streams,
ame_stream_create_cu_range), through the C-ABI.

Kind 24 is kind 22 with six GEMV worker workgroups per slice instead of seven
(7 workgroups per slice: BASELINE config 5's 32 slices hold 224 CUs), a worker
wave holding 176 nodes (152 in registers, 24 in LDS).  Checks:

* kind resolution, its capacity (n <= 6 x 4 x 176) and co-residency limit;
* the fp64 oracle at small shapes, good / bad / naive, r = 32 and smaller r
  (tolerances of tests/test_gpu_large.py);
* config 5's rank shape (n = 4096, T = 32, r = 32): the second sweep's first
  600 nodes of all 32 slices against the fp64 oracle;
* elbo_cus: the ELBO kernels on CUs [0, 32), the sweep on the other 224 --
  the fit (means, covariances, every iteration's ELBO and MSE) bit for bit
  the single-stream run, at config 5's rank shape and at a small shape;
  bad CU ranges and kinds are refused;
* elbo_first (opt-in: the ELBO queued before the speculative sweep): bit for
  bit the default sweep-first order.

Reference: structured_mf.py:211-326, naive_mf.py:207-282, temporal_ame.py:255-291.
"""
import ctypes

import numpy as np
import pytest
import torch

from test_gpu_large import _check_vs_oracle, _params, _vi

pytestmark = pytest.mark.gpu

W6 = 24   # _lib.AME_SWEEP_V2_W6


def _kind(n, T, r, request=0, variant=0):
    from ame_amd import _lib
    L = _lib.lib()
    d = _lib.ame_dims(n, r, T, 0, T, variant)
    return int(L.ame_sweep_kind(ctypes.byref(d), request))


def test_w6_kind_resolution(gpu_device):
    from ame_amd import _lib
    L = _lib.lib()
    assert _lib.AME_SWEEP_V2_W6 == W6
    assert _kind(4096, 32, 32, W6) == W6
    assert L.ame_sweep_orders_slices(4096, 32, W6) == 0
    cus = torch.cuda.get_device_properties(gpu_device).multi_processor_count
    cap = int(L.ame_sweep_max_slices(4096, 32, W6))
    assert cap == cus // 7
    assert _kind(4096, cap, 32, W6) == W6
    assert _kind(4096, cap + 1, 32, W6) == -1     # refused, not re-routed
    assert _kind(4224, 4, 32, W6) == W6
    assert _kind(4300, 4, 32, W6) == -1           # n > 6 x 4 x 176 worker slots


@pytest.mark.parametrize("n,T,r,method,lr", [
    (24, 3, 32, "good", 0.5), (20, 4, 32, "bad", 1.0), (22, 3, 32, "naive", 0.3),
    (2, 2, 32, "good", 1.0), (301, 4, 32, "good", 0.5), (130, 3, 24, "naive", 0.5),
    (64, 3, 8, "good", 0.5)])
def test_w6_vs_oracle(n, T, r, method, lr, gpu_device):
    vi = _check_vs_oracle(n, T, r, method, lr, gpu_device, sweep_kernel=W6)
    assert vi.engine.sweep_kind == W6 and not vi.engine.pipelined


def _fit(n, T, r, method, lr, dev, iters, seed, **opts):
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(n, T, r, seed=seed)
    m.generate_data_fast(device=dev, seed=seed + 1)
    vi = _vi(m, method, lr, dev, **opts)
    h = vi.fit(max_iter=iters, tolerance=0.0, verbose=False)
    out = (vi.engine.means_local().cpu().numpy(), vi.engine.covs_local()[:64].cpu().numpy(),
           [float(e) for e in h["elbo"]], [float(e) for e in h["reconstruction_error"]])
    eng = vi.engine
    return eng, out


@pytest.mark.parametrize("n,T,r,method,iters", [(300, 6, 32, "good", 4), (200, 5, 24, "naive", 3)])
def test_elbo_cus_small_bit_equal(n, T, r, method, iters, gpu_device):
    from ame_amd import _lib
    eng, a = _fit(n, T, r, method, 0.4, gpu_device, iters, 5, sweep_kernel=W6, elbo_cus=32)
    assert eng.elbo_stream is not None and eng.sweep_kind == W6
    del eng
    _, b = _fit(n, T, r, method, 0.4, gpu_device, iters, 5, sweep_kernel=W6)
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    # kind 22 too (8 workgroups per slice)
    eng, c = _fit(n, T, r, method, 0.4, gpu_device, iters, 5,
                  sweep_kernel=_lib.AME_SWEEP_V2_WORKERS, elbo_cus=16)
    assert eng.elbo_stream is not None
    del eng
    _, d = _fit(n, T, r, method, 0.4, gpu_device, iters, 5, sweep_kernel=_lib.AME_SWEEP_V2_WORKERS)
    for x, y in zip(c, d):
        assert np.array_equal(np.asarray(x), np.asarray(y))


@pytest.mark.parametrize("n,T,r,method,iters", [(300, 6, 32, "good", 4), (200, 5, 24, "naive", 3)])
def test_elbo_first_bit_equal(n, T, r, method, iters, gpu_device):
    """The ELBO queued before the speculative sweep (elbo_first, opt-in)
    changes only the launch order: the fit bit for bit the default sweep-first
    order, for kind 22 and kind 24."""
    from ame_amd import _lib
    for kind in (_lib.AME_SWEEP_V2_WORKERS, W6):
        eng, a = _fit(n, T, r, method, 0.4, gpu_device, iters, 7, sweep_kernel=kind,
                      elbo_first=True)
        assert eng.elbo_first and eng.sweep_kind == kind
        del eng
        eng, b = _fit(n, T, r, method, 0.4, gpu_device, iters, 7, sweep_kernel=kind)
        assert not eng.elbo_first
        del eng
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x), np.asarray(y))


def test_elbo_cus_refused(gpu_device):
    from ame_amd import TemporalAMEModel, _lib
    L = _lib.lib()
    p = ctypes.c_void_p()
    cus = torch.cuda.get_device_properties(gpu_device).multi_processor_count
    assert L.ame_stream_create_cu_range(0, 0, ctypes.byref(p)) != 0
    assert L.ame_stream_create_cu_range(cus - 4, 8, ctypes.byref(p)) != 0
    assert L.ame_stream_create_cu_range(-1, 4, ctypes.byref(p)) != 0
    assert L.ame_stream_create_cu_range(cus - 8, 8, ctypes.byref(p)) == 0 and p.value
    assert L.ame_stream_destroy(p) == 0
    m = TemporalAMEModel(40, 3, 32, seed=1)
    m.generate_data_fast(device=gpu_device, seed=2)
    with pytest.raises(ValueError):
        _vi(m, "good", 0.5, gpu_device, elbo_cus=32).engine                      # AUTO kernel
    with pytest.raises(ValueError):
        _vi(m, "good", 0.5, gpu_device, sweep_kernel=W6, elbo_cus=cus).engine   # no CUs left


@pytest.mark.timeout(600)
def test_config5_rank_shape_w6_and_elbo_cus(gpu_device):
    """BASELINE config 5's per-rank shape on kind 24: the in-order run's
    second sweep (first 600 nodes of all 32 slices) against the fp64 oracle,
    and the elbo_cus schedule (ELBO on 32 CUs beside the sweep on 224) bit for
    bit the single-stream run over 3 iterations."""
    import ame_oracle as O
    from ame_amd import TemporalAMEModel
    n, T, r, lr, KF = 4096, 32, 32, 0.01, 600

    def model():
        m = TemporalAMEModel(n, T, r, seed=42)
        m.generate_data_fast(device=gpu_device, seed=42)
        return m

    vi = _vi(model(), "good", lr, gpu_device, sweep_kernel=W6, elbo_cus=32)
    assert vi.engine.sweep_kind == W6 and len(vi.engine.groups) == 1
    h = vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    prod = (vi.engine.means_local().cpu().numpy(), vi.engine.covs_local()[:KF].cpu().numpy(),
            [float(e) for e in h["elbo"]])
    del vi
    torch.cuda.empty_cache()
    m = model()
    vi = _vi(m, "good", lr, gpu_device, sweep_kernel=W6)
    eng = vi.engine
    vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    x1 = eng.means_local().cpu().numpy().astype(np.float64)
    c1 = eng.covs_local()[:KF].cpu().numpy().astype(np.float64)
    vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    got_m = eng.means_local().cpu().numpy()
    got_c = eng.covs_local()[:KF].cpu().numpy()
    h3 = vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    assert np.array_equal(eng.means_local().cpu().numpy(), prod[0])
    assert np.array_equal(eng.covs_local()[:KF].cpu().numpy(), prod[1])
    assert [float(e) for e in h3["elbo"]] == prod[2]   # (the history accumulates over fit calls)
    YK = m.Y[:KF].cpu().numpy()
    del vi, eng
    torch.cuda.empty_cache()
    O.sweep_stats(YK, x1, c1, _params(m), "good", lr, nodes=range(KF))
    err = np.abs(got_m[:KF].astype(np.float64) - x1[:KF]).max()
    cerr = np.abs(got_c.astype(np.float64) - c1).max()
    print(f"config 5 rank shape, kind 24: nodes 0..{KF - 1} vs fp64 oracle: max|dmean| "
          f"{err:.3e} (max|mean| {np.abs(x1[:KF]).max():.3f}), max|dcov| {cerr:.3e}")
    assert err <= 5e-6 * max(1.0, np.abs(x1[:KF]).max()), err
    assert cerr <= 1e-6 * max(1.0, np.abs(c1).max()), cerr
