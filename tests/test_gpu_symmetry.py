"""Damped covariances are exactly symmetric on every sweep kernel.

The reference symmetrises each new covariance ((C + C^T) / 2,
structured_mf.py:274-282) and damps elementwise in fp32
(lr * C_new + (1 - lr) * C_old, structured_mf.py:283-287), so X_cov[i, t] is
bit-symmetric.  The kernels compute the lower triangle once and damp the entry
and its mirror with the same products and sum (mul_add_rn, no FMA contraction);
a contracted form rounded the two halves differently.
"""
import numpy as np
import pytest

from test_gpu_large import _vi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,T,r,method,kind", [
    (64, 4, 32, "good", 22), (64, 4, 32, "bad", 22), (64, 4, 32, "naive", 22),
    (1024, 8, 16, "good", 3), (256, 8, 16, "bad", 3), (256, 8, 16, "naive", 3),
    (48, 3, 8, "good", 20), (48, 3, 8, "good", 21)])
def test_cov_exactly_symmetric(n, T, r, method, kind, gpu_device):
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(n, T, r, seed=2)
    m.generate_data_fast(seed=3)
    vi = _vi(m, method, 0.7, gpu_device, sweep_kernel=kind)
    assert vi.engine.sweep_kind == kind
    vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    C = vi.X_cov.numpy()
    asym = np.argwhere(C != np.swapaxes(C, -1, -2))
    if len(asym):
        # diagnostics for a recurrence (seen once in a full-suite run, not
        # reproduced in 12 repetitions): magnitude, and whether the
        # in-order schedule of the same fit agrees
        m2 = TemporalAMEModel(n, T, r, seed=2)
        m2.generate_data_fast(seed=3)
        v2 = _vi(m2, method, 0.7, gpu_device, sweep_kernel=kind, pipeline=False, speculate=False)
        v2.fit(max_iter=2, tolerance=0.0, verbose=False)
        C2 = v2.X_cov.numpy()
        print("asymmetric entries", len(asym), "max", np.abs(C - np.swapaxes(C, -1, -2)).max(),
              "in-order run asymmetric", np.count_nonzero(C2 != np.swapaxes(C2, -1, -2)),
              "max |C - C_inorder|", np.abs(C - C2).max(),
              "max |mean - mean_inorder|", np.abs(vi.X_mean.numpy() - v2.X_mean.numpy()).max())
    assert len(asym) == 0, (len(asym), asym[:5].tolist())
