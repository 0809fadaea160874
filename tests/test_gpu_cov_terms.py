"""GPU parity of the covariance-terms kernel (K2, `ame_cov` through the C-ABI)
against numpy fp64 on the same fp32 covariances.

Per stored covariance S (d x d, fp32): log|S| with torch.logdet semantics
(-inf for a zero determinant, nan for a negative one), tr S, tr(Q^-1 S) for
t >= 1 and tr(S0^-1 S) at t = 0 (structured_mf.py:142-144, :166, :193,
:202-209).  Both kernel forms are covered: the column-per-lane LDL^T (r below
AME_COV_MFMA_MIN_R) and the MFMA blocked LDL^T (r >= it; padded to 16 x 16
tiles when 2r is not a multiple of 16), on random well-conditioned SPD
covariances, slices with and without t = 0 (t_begin 0 / 1), indefinite ones
(negative determinant in the complement or in the (a,b) block) and the
config-5 size (r = 32) on a slice sample.  fp64 throughout, so the bound is
1e-10 relative (LDL^T without pivoting vs numpy's LU).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _spd(rng, m, d, cond=4.0):
    X = rng.standard_normal((m, d, 2 * d))
    S = X @ X.transpose(0, 2, 1) / (2 * d) + np.eye(d) / cond
    return S


def _run(cov32, consts, n, T, t_begin, r, dev):
    from ame_amd import _lib
    L = _lib.lib()
    d = 2 + 2 * r
    cov = torch.from_numpy(cov32.reshape(-1)).to(dev)
    cst = torch.from_numpy(consts.reshape(-1)).to(dev)
    out = torch.full((T * n * 4,), 7.0, dtype=torch.float64, device=dev)
    dims = _lib.ame_dims(n, r, T, t_begin, t_begin + T, 0)
    args = _lib.ame_cov_args(cov=cov.data_ptr(), consts=cst.data_ptr(), cov_terms=out.data_ptr())
    torch.cuda.synchronize()
    _lib.check(L.ame_cov(ctypes.byref(dims), ctypes.byref(args), None), "ame_cov")
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(T, n, 4)


def _ref(cov32, consts, t_begin):
    C = cov32.astype(np.float64)            # (T, n, d, d)
    T = C.shape[0]
    sign, lad = np.linalg.slogdet(C)
    ld = np.where(sign > 0, lad, np.where(sign == 0, -np.inf, np.nan))
    tr = np.trace(C, axis1=-2, axis2=-1)
    S0i, Qi = consts[0], consts[1]
    tq = np.einsum("ab,tnba->tn", Qi, C)
    t0 = np.einsum("ab,tnba->tn", S0i, C)
    tg = t_begin + np.arange(T)[:, None]
    return np.stack([ld, tr, np.where(tg >= 1, tq, 0.0), np.where(tg == 0, t0, 0.0)], axis=-1)


def _consts(rng, d):
    c = np.zeros((5, d, d))
    for k in range(2):
        M = _spd(rng, 1, d)[0]
        c[k] = np.linalg.inv(M)
        c[k] = 0.5 * (c[k] + c[k].T)
    return c


def _check(got, ref):
    fin = np.isfinite(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), (got[..., 0], ref[..., 0])
    assert np.array_equal(np.isneginf(got), np.isneginf(ref))
    err = np.abs(got[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))
    assert err.max() <= 1e-10, err.max()


@pytest.mark.parametrize("r", [1, 3, 8, 12, 16, 20, 24, 28, 32])
@pytest.mark.parametrize("t_begin", [0, 1])
def test_cov_terms_random_spd(r, t_begin, gpu_device):
    rng = np.random.default_rng(100 + r + 7 * t_begin)
    n, T = 37, 3
    d = 2 + 2 * r
    cov = _spd(rng, T * n, d).reshape(T, n, d, d).astype(np.float32)
    consts = _consts(rng, d)
    got = _run(cov, consts, n, T, t_begin, r, gpu_device)
    _check(got, _ref(cov, consts, t_begin))


@pytest.mark.parametrize("r", [4, 16, 24, 32])
def test_cov_terms_indefinite(r, gpu_device):
    """Negative determinants (one negative eigenvalue in the complement, or a
    negative-determinant (a,b) block): nan, as torch.logdet."""
    rng = np.random.default_rng(7 + r)
    n, T = 24, 2
    d = 2 + 2 * r
    S = _spd(rng, T * n, d)
    for m in range(0, T * n, 3):   # every third: a negative eigenvalue
        w, V = np.linalg.eigh(S[m])
        w[(m // 3) % d] = -0.5 - m * 0.01
        S[m] = (V * w) @ V.T
    S[1, :2, :2] = [[1.0, 2.0], [2.0, 1.0]]   # (a,b) block with det < 0 (S indefinite)
    cov = S.reshape(T, n, d, d).astype(np.float32)
    consts = _consts(rng, d)
    got = _run(cov, consts, n, T, 0, r, gpu_device)
    ref = _ref(cov, consts, 0)
    assert np.isnan(ref[..., 0]).sum() >= T * n // 3
    _check(got, ref)


def test_cov_terms_config5_sample(gpu_device):
    """Config 5's rank shape (n = 4096, r = 32) on two slices, the first one
    t = 0: every covariance of both slices against numpy."""
    rng = np.random.default_rng(5)
    n, T, r = 4096, 2, 32
    d = 2 + 2 * r
    cov = _spd(rng, T * n, d, cond=2.0).reshape(T, n, d, d).astype(np.float32)
    consts = _consts(rng, d)
    got = _run(cov, consts, n, T, 0, r, gpu_device)
    _check(got, _ref(cov, consts, 0))
