"""CPU: the loop-structured restatement (oracle/ame_loop_oracle.py, the
§8d(i) reference-shaped CPU baseline) agrees with the vectorised oracle, which
is itself pinned to the reference's golden fixtures."""
import numpy as np
import pytest
import torch

import ame_loop_oracle as LO
import ame_oracle as O


def _problem(n=9, T=4, r=2, seed=3):
    rng = np.random.default_rng(seed)
    p = O.model_params(r)
    d = 2 + 2 * r
    Y = rng.standard_normal((n, n, T, 2)).astype(np.float32)
    Xm = (0.3 * rng.standard_normal((n, T, d))).astype(np.float32)
    Xc = np.broadcast_to(0.5 * np.eye(d, dtype=np.float32), (n, T, d, d)).copy()
    return p, Y, Xm, Xc


@pytest.mark.parametrize("variant", ["good", "bad", "naive"])
def test_loop_update_matches_vectorised(variant):
    p, Y, Xm, Xc = _problem()
    Xm_t, Xc_t = torch.from_numpy(Xm.copy()), torch.from_numpy(Xc.copy())
    Y_t = torch.from_numpy(Y)
    cons = O.prior_terms(p, Xm.shape[1], np.float32)
    for i in range(3):
        O.update_node(Y, Xm, Xc, p, i, variant, 0.5, cons)
        LO.update_node_loop(Y_t, Xm_t, Xc_t, p, i, variant, 0.5)
    assert np.abs(Xm_t.numpy() - Xm).max() < 2e-5
    assert np.abs(Xc_t.numpy() - Xc).max() < 2e-5


@pytest.mark.parametrize("variant", ["good", "naive"])
def test_loop_loglik_matches_vectorised(variant):
    p, Y, Xm, Xc = _problem()
    T = Xm.shape[1]
    ref = O.expected_loglik(Y, Xm, Xc, p, variant)
    got = sum(float(LO.loglik_pairs_loop(torch.from_numpy(Y), torch.from_numpy(Xm),
                                         torch.from_numpy(Xc), p, variant, t)) for t in range(T))
    assert abs(got - ref) <= 1e-5 * abs(ref)
