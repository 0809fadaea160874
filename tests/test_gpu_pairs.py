"""ELBO pair kernel v2 (LDS-DMA Y stream, ame_elbo.hip ame_pairs2_kernel)
against the register-streaming v1 kernel and the fp64 oracle, at even and
odd n (Yt rows are padded to even length, so v2 runs at any n).

Reference: structured_mf.py:124-150 (expected log-likelihood),
temporal_ame.py:255-291 (reconstruction error).  v2 is the default at every
n; engine option pairs_kernel=AME_PAIRS_V1 selects v1.  Both form the same fp32 products and per-tile fp32
partial sums, so they agree to a few fp32 ulps of the total (bound 1e-6
relative, stated here); against the fp64 oracle the ELBO log-likelihood and
the reconstruction error are held to 5e-6 relative, as in test_gpu_parity.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sums(vi, v1):
    from ame_amd import _lib
    eng = vi.engine
    eng.options.pairs_kernel = _lib.AME_PAIRS_V1 if v1 else _lib.AME_PAIRS_V2
    eng.invalidate()
    eng.launch_elbo()
    out = eng.out.cpu().numpy().astype(np.float64).copy()
    eng._check_status()
    return out


@pytest.mark.parametrize("n,T,r,swap", [
    (64, 3, 16, True), (130, 2, 16, True), (200, 3, 8, False), (256, 4, 32, True),
    (1024, 8, 16, True), (1024, 2, 16, False), (2, 3, 1, True), (98, 2, 5, True),
    (192, 5, 3, False), (4096, 1, 32, True),
    # odd n: rows padded to even length (ame_ystride), the v2 kernel's DMA
    # chunks stay 16-byte aligned and the pad column is masked
    (97, 3, 5, True), (257, 2, 16, False), (1023, 2, 16, True), (3, 2, 2, True)])
def test_pairs_v2_matches_v1_and_oracle(n, T, r, swap, gpu_device):
    import ame_oracle as O
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    m = TemporalAMEModel(n, T, r, seed=5)
    m.generate_data_fast(seed=9)
    if not swap:
        m.Y[1, n - 1, 0, 0] += 0.75
        m.Y[n - 2, 0, T - 1, 1] -= 0.5
    vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=0.3, device=gpu_device)
    assert vi.engine.swap_consistent == swap
    vi.fit(max_iter=1, tolerance=0.0, verbose=False)   # a non-initial state
    a = _sums(vi, v1=True)
    b = _sums(vi, v1=False)
    # out[0] = sum of the quadratic form over i<j, out[7] = squared-error sum
    for k in (0, 7):
        assert abs(b[k] - a[k]) <= 1e-6 * abs(a[k]), (k, a[k], b[k])
    if n <= 1024:
        Y = m.Y.numpy().astype(np.float64)
        X = vi.X_mean.numpy().astype(np.float64)
        rinv = m.R_inv.numpy().astype(np.float64)
        iu, ju = np.triu_indices(n, k=1)
        off = ~np.eye(n, dtype=bool)
        quad = sq = 0.0
        for t in range(T):   # the sums behind expected_loglik and recon_error
            mu = O.compute_mean(X[:, t], r)
            res = Y[iu, ju, t, :] - mu[iu, ju]
            quad += float(np.einsum("pa,ab,pb->", res, rinv, res))
            sq += float(((Y[:, :, t] - mu) ** 2)[off].sum())
        assert abs(b[0] - quad) <= 5e-6 * abs(quad), (b[0], quad)
        assert abs(b[7] - sq) <= 5e-6 * abs(sq), (b[7], sq)
