"""GPU parity of the v2 sweep's wide and large modes, through the C-ABI:

* r = 32 (d = 66 > 64: two state rows per solver lane), BASELINE config 5's
  latent dim, against the fp64 oracle on small problems, all three variants;
* the slice's (U,V) block read from HBM instead of LDS (kind AME_SWEEP_V2_HBM
  requested at small n; automatic at n = 3400);
* config 5's node count and latent dim (n = 4096, r = 32) on a few slices:
  the first nodes of the Gauss-Seidel sweep against the oracle replaying the
  same sweep prefix (node i depends only on the initial state and on nodes < i,
  Appendix B of SURVEY.md), and the ELBO / MSE of the device state against the
  oracle's ELBO of that same state.

Tolerances as in test_gpu_parity.py: 5e-6 relative vs the fp64 oracle, or no
further from it than the reference's own fp32 arithmetic (fp32 oracle) is.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PKEYS = ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")


def _vi(model, method, lr, dev, **opts):
    from ame_amd import TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    if method == "naive":
        return TemporalAMENaiveMFVI(model, learning_rate=lr, device=dev, engine_options=opts)
    return TemporalAMEStructuredMFVI(model, factorization=method, learning_rate=lr, device=dev,
                                     engine_options=opts)


def _params(m, dtype=np.float64):
    return {k: getattr(m, k).numpy().astype(dtype) for k in PKEYS}


def _check_vs_oracle(n, T, r, method, lr, dev, iters=2, **opts):
    import ame_oracle as O
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(n, T, r, seed=7)
    m.generate_data_fast(seed=11)
    vi = _vi(m, method, lr, dev, **opts)
    Xm = vi.X_mean.numpy().astype(np.float64).copy()
    Xc = vi.X_cov.numpy().astype(np.float64).copy()
    Xm32, Xc32 = vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()
    params = _params(m)
    ref = O.fit(m.Y.numpy().astype(np.float64), Xm, Xc, params, method, lr, iters, 0.0)
    O.fit(m.Y.numpy(), Xm32, Xc32, _params(m, np.float32), method, lr, iters, 0.0)
    fp32_err = np.abs(Xm32.astype(np.float64) - Xm).max()
    h = vi.fit(max_iter=iters, tolerance=0.0, verbose=False)
    err = np.abs(vi.X_mean.numpy() - Xm).max()
    # fp32 allowance: the kernel's error may exceed the fp32 restatement's own
    # deviation from fp64 by the measured rounding-order spread plus a margin.
    # Two fp32 evaluations that differ only in rounding order land on either
    # side of each other: measured ratios err / fp32_err were 0.56 (damping
    # FMA-contracted), 1.11 (rounded as the reference does) on (64, 3, 8, good,
    # 0.5) and 1.31 on kind 20 (tools/parity_margin.py); the bound
    # is 1.5x, and every case prints its ratio
    ratio = err / fp32_err if fp32_err > 0 else 0.0
    print(f"parity {n}x{T} r={r} {method}: err {err:.3e}, fp32 restatement {fp32_err:.3e}, "
          f"ratio {ratio:.2f}")
    assert err <= max(5e-6 * max(1.0, np.abs(Xm).max()), 1.5 * fp32_err), (err, fp32_err, ratio)
    cerr = np.abs(vi.X_cov.numpy() - Xc).max()
    assert cerr <= 1e-6 * max(1.0, np.abs(Xc).max()), cerr
    for a, b in zip(h["elbo"], ref["elbo"]):
        assert abs(float(a) - b) <= 5e-6 * abs(b), (float(a), b)
    for a, b in zip(h["reconstruction_error"], ref["reconstruction_error"]):
        assert abs(a - b) <= 5e-6 * abs(b), (a, b)
    return vi


@pytest.mark.parametrize("n,T,r,method,lr", [
    (24, 3, 32, "good", 0.5), (20, 4, 32, "bad", 1.0), (22, 3, 32, "naive", 0.3),
    (2, 2, 32, "good", 1.0), (40, 1, 32, "good", 0.01)])
def test_r32_vs_oracle(n, T, r, method, lr, gpu_device):
    """d = 66: the solver wave holds rows 64, 65 in a second register set."""
    vi = _check_vs_oracle(n, T, r, method, lr, gpu_device)
    assert vi.engine.r == 32


@pytest.mark.parametrize("n,T,r,method,lr", [
    (50, 4, 4, "good", 0.5), (37, 3, 5, "bad", 1.0), (45, 3, 16, "naive", 0.7),
    (30, 3, 32, "good", 0.5), (700, 2, 16, "good", 0.5)])
def test_global_slice_vs_oracle(n, T, r, method, lr, gpu_device):
    """(U,V) block in HBM on the single-workgroup v2 sweep (kind 21 requested)."""
    from ame_amd import _lib
    vi = _check_vs_oracle(n, T, r, method, lr, gpu_device, sweep_kernel=_lib.AME_SWEEP_V2_HBM)
    assert vi.engine.sweep_kind == _lib.AME_SWEEP_V2_HBM


@pytest.mark.parametrize("n,T,r,method,lr", [(64, 5, 8, "good", 0.5), (33, 4, 3, "bad", 1.0)])
def test_v2_lds_slice_vs_oracle(n, T, r, method, lr, gpu_device):
    """The single-workgroup v2 sweep with the slice in LDS (kind 20)."""
    from ame_amd import _lib
    vi = _check_vs_oracle(n, T, r, method, lr, gpu_device, sweep_kernel=_lib.AME_SWEEP_V2_LDS)
    assert vi.engine.sweep_kind == _lib.AME_SWEEP_V2_LDS


def test_auto_global_slice_past_v3(gpu_device):
    """n = 3400, r = 16: past the v3 sweep's register/LDS budget and past the v2
    LDS slice, so the v2 sweep keeps the slice in HBM on its own."""
    from ame_amd import _lib
    vi = _check_vs_oracle(3400, 1, 16, "good", 0.5, gpu_device, iters=1,
                          sweep_kernel=_lib.AME_SWEEP_V2_SINGLE)
    assert vi.engine.sweep_kind == _lib.AME_SWEEP_V2_HBM   # past v3 and the LDS slice
    assert _lib.lib().ame_sweep_orders_slices(3400, 16, vi.engine.sweep_kind) == 0


@pytest.mark.parametrize("method", ["good", "bad", "naive"])
def test_config5_shape_prefix_and_elbo(method, gpu_device):
    """n = 4096, r = 32 (config 5), 3 slices: the first 3 nodes of one sweep
    against the oracle's replay of the same prefix, and the device ELBO / MSE
    against the oracle's ELBO of the device state."""
    import ame_oracle as O
    from ame_amd import TemporalAMEModel
    n, T, r, lr, k = 4096, 3, 32, 0.5, 3
    m = TemporalAMEModel(n, T, r, seed=5)
    m.generate_data_fast(seed=6)
    vi = _vi(m, method, lr, gpu_device)
    assert not vi.engine.pipelined   # v2 sweep with the slice in HBM
    Y64 = m.Y.numpy().astype(np.float64)
    Y32 = m.Y.numpy()
    Xm = vi.X_mean.numpy().astype(np.float64).copy()
    Xc = vi.X_cov.numpy().astype(np.float64).copy()
    Xm32, Xc32 = vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()
    p64, p32 = _params(m), _params(m, np.float32)
    c64, c32 = O.prior_terms(p64, T, np.float64), O.prior_terms(p32, T, np.float32)
    for i in range(k):
        O.update_node(Y64, Xm, Xc, p64, i, method, lr, c64)
        O.update_node(Y32, Xm32, Xc32, p32, i, method, lr, c32)
    h = vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    got_m = vi.X_mean.numpy()[:k].astype(np.float64)
    got_c = vi.X_cov.numpy()[:k].astype(np.float64)
    fp32_err = np.abs(Xm32[:k].astype(np.float64) - Xm[:k]).max()
    err = np.abs(got_m - Xm[:k]).max()
    assert err <= max(5e-6 * max(1.0, np.abs(Xm[:k]).max()), fp32_err), (err, fp32_err)
    cerr = np.abs(got_c - Xc[:k]).max()
    assert cerr <= 1e-6 * max(1.0, np.abs(Xc[:k]).max()), cerr
    # ELBO / MSE kernels at full size on the device's own post-sweep state
    Sm = vi.X_mean.numpy()
    Sc = vi.X_cov.numpy()
    e_ref = O.elbo(Y64, Sm, Sc, p64, method)
    mse_ref = O.recon_error(Y64, Sm)
    assert np.isfinite(float(h["elbo"][0]))
    assert abs(float(h["elbo"][0]) - e_ref) <= 5e-6 * abs(e_ref), (float(h["elbo"][0]), e_ref)
    assert abs(h["reconstruction_error"][0] - mse_ref) <= 5e-6 * mse_ref
