"""GPU: the v4 sweep (MFMA block GEMM for the observation term,
csrc/ame_sweep4.hip) against the fp64 oracle, and against the v3 sweep
(per-step GEMV, the default) on the same problems.

v4 is opt-in (AME_SWEEP_V4=1; v3 is the default) for r <= 16,
n % 4 == 0, 8 <= n <= 2048;
the cases cover block and window edges: n < 16 (one block), n not a multiple
of 16 (partial last block, padded columns), n = 2048 (two column groups per
GEMM wave and step), r < 16 (padded MFMA columns) and all three variants.
Tolerances as tests/test_gpu_parity.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _force_v4(monkeypatch):
    monkeypatch.setenv("AME_SWEEP_V4", "1")


def _vi(model, method, lr, dev):
    from ame_amd import TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    if method == "naive":
        return TemporalAMENaiveMFVI(model, learning_rate=lr, device=dev)
    return TemporalAMEStructuredMFVI(model, factorization=method, learning_rate=lr, device=dev)


def _params(m, dtype=np.float64):
    return {k: getattr(m, k).cpu().numpy().astype(dtype) for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")}


@pytest.mark.parametrize("n,T,r,method,lr", [
    (8, 3, 2, "good", 1.0), (12, 4, 3, "bad", 0.7), (20, 5, 4, "naive", 0.5),
    (36, 6, 16, "good", 0.5), (100, 5, 8, "good", 1.0), (148, 3, 5, "bad", 0.5),
    (260, 3, 16, "naive", 0.3), (1000, 2, 16, "good", 0.5), (2048, 1, 16, "good", 0.3),
    (64, 9, 12, "good", 0.01), (96, 4, 1, "good", 1.0)])
def test_sweep4_vs_oracle(n, T, r, method, lr, gpu_device):
    import ame_oracle as O
    from ame_amd import TemporalAMEModel, _lib
    assert _lib.lib().ame_sweep_orders_slices(n, r) == 1
    m = TemporalAMEModel(n, T, r, seed=17)
    m.generate_data_fast(seed=19)
    vi = _vi(m, method, lr, gpu_device)
    Xm = vi.X_mean.numpy().astype(np.float64).copy()
    Xc = vi.X_cov.numpy().astype(np.float64).copy()
    Xm32, Xc32 = vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()
    ref = O.fit(m.Y.numpy().astype(np.float64), Xm, Xc, _params(m), method, lr, 2, 0.0)
    O.fit(m.Y.numpy(), Xm32, Xc32, _params(m, np.float32), method, lr, 2, 0.0)
    fp32_err = np.abs(Xm32.astype(np.float64) - Xm).max()
    h = vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    err = np.abs(vi.X_mean.numpy() - Xm).max()
    assert err <= max(5e-6 * max(1.0, np.abs(Xm).max()), fp32_err), (err, fp32_err)
    cerr = np.abs(vi.X_cov.numpy() - Xc).max()
    assert cerr <= 1e-6 * max(1.0, np.abs(Xc).max()), cerr
    for a, b in zip(h["elbo"], ref["elbo"]):
        assert abs(float(a) - b) <= 5e-6 * abs(b), (float(a), b)
    for a, b in zip(h["reconstruction_error"], ref["reconstruction_error"]):
        assert abs(a - b) <= 5e-6 * abs(b), (a, b)


def test_sweep4_matches_v3(gpu_device, monkeypatch):
    """Same problem through v4 and v3: means agree to fp32 round-off."""
    from ame_amd import TemporalAMEModel
    out = []
    for v4 in ("1", "0"):
        monkeypatch.setenv("AME_SWEEP_V4", v4)
        m = TemporalAMEModel(256, 16, 8, seed=3)
        m.generate_data_fast(seed=3)
        vi = _vi(m, "good", 0.5, gpu_device)
        h = vi.fit(max_iter=3, tolerance=0.0, verbose=False)
        out.append((vi.X_mean.numpy().copy(), [float(e) for e in h["elbo"]]))
    d = np.abs(out[0][0] - out[1][0]).max()
    assert d <= 2e-5 * max(1.0, np.abs(out[1][0]).max()), d
    assert np.allclose(out[0][1], out[1][1], rtol=2e-6, atol=0)
