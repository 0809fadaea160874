"""tests/elbo_check.py (batched torch-CPU ELBO / MSE for the large-shape GPU
tests) equals the numpy oracle's ELBO split and MSE (CPU only)."""
import numpy as np
import pytest

import ame_oracle as O
from elbo_check import elbo_and_mse


@pytest.mark.parametrize("n,T,r,variant", [(30, 4, 3, "good"), (17, 1, 2, "naive"),
                                           (24, 5, 32, "bad")])
def test_matches_oracle(n, T, r, variant):
    rng = np.random.default_rng(n + T + r)
    d = 2 + 2 * r
    Y = rng.standard_normal((n, n, T, 2)).astype(np.float32)
    Xm = (0.3 * rng.standard_normal((n, T, d))).astype(np.float32)
    A = rng.standard_normal((n, T, d, d)) * 0.1
    Xc = (A @ np.swapaxes(A, -1, -2) + 0.5 * np.eye(d)).astype(np.float32)
    p = {k: v.astype(np.float64) for k, v in O.model_params(r).items()}
    got = elbo_and_mse(Y, Xm, Xc, p, variant)
    ref = O.elbo_split(Y, Xm, Xc, p, variant)
    for k, v in zip(("loglik", "prior0", "trans", "entropy"), ref):
        assert abs(got[k] - v) <= 1e-10 * max(1.0, abs(v)), (k, got[k], v)
    assert abs(got["recon"] - O.recon_error(Y, Xm)) <= 1e-12
