"""Host-side drop-in behaviour (no GPU): model generator and VI initialisation
are bit-identical to the reference; constructor/getter/fit-loop semantics
mirror src/inference/base.py and tests/test_inference.py of the reference.
"""
import numpy as np
import pytest
import torch

from conftest import golden

CFG = {"c1": (15, 10, 2), "tfix": (10, 5, 2), "mid": (40, 12, 3)}


@pytest.mark.parametrize("tag", list(CFG))
def test_generator_bit_exact(tag):
    from ame_amd import TemporalAMEModel
    n, T, r = CFG[tag]
    m = TemporalAMEModel(n, T, r, ar_coefficient=0.8, rho_dyadic=0.5, seed=42)
    Y, X = m.generate_data(return_latents=True)
    z = golden(f"{tag}_model.npz")
    assert np.array_equal(Y.numpy(), z["Y"])
    assert np.array_equal(X.numpy(), z["X_true"])
    for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q"):
        assert np.array_equal(getattr(m, k).numpy(), z[k]), k
    assert (m.n, m.T, m.r, m.d) == (n, T, r, 2 + 2 * r)


@pytest.mark.parametrize("tag,method", [("c1", "good"), ("c1", "bad"), ("c1", "naive"),
                                        ("mid", "good"), ("mid", "bad"), ("tfix", "naive")])
def test_init_bit_exact(tag, method):
    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    import glob
    import os
    from conftest import GOLDEN
    n, T, r = CFG[tag]
    m = TemporalAMEModel(n, T, r, seed=42)
    m.generate_data()
    f = sorted(glob.glob(os.path.join(GOLDEN, f"{tag}_{method}_lr*.npz")))[0]
    z = np.load(f)
    lr = float(z["lr"])
    if method == "naive":
        vi = TemporalAMENaiveMFVI(m, learning_rate=lr)
    else:
        vi = TemporalAMEStructuredMFVI(m, factorization=method, learning_rate=lr)
    assert np.array_equal(vi.X_mean.numpy(), z["init_mean"])
    assert np.array_equal(vi.X_cov.numpy(), z["init_cov"])


@pytest.fixture
def temporal_model():
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(n_nodes=10, n_time=5, latent_dim=2, ar_coefficient=0.8, seed=42)
    m.generate_data(return_latents=True)
    return m


def test_structured_init_api(temporal_model):
    """test_inference.py:114-154 of the reference (init structure, ValueError)."""
    from ame_amd import TemporalAMEStructuredMFVI
    m = temporal_model
    vi = TemporalAMEStructuredMFVI(m, factorization="good")
    assert (vi.n, vi.T, vi.d, vi.factorization, vi.lr) == (m.n, m.T, m.d, "good", 1.0)
    assert vi.X_mean.shape == (m.n, m.T, m.d)
    assert vi.X_cov.shape == (m.n, m.T, m.d, m.d)
    off = vi.X_cov - torch.diag_embed(torch.diagonal(vi.X_cov, dim1=-2, dim2=-1))
    assert (off.abs().amax(dim=(-1, -2)) > 0).all()
    bad = TemporalAMEStructuredMFVI(m, factorization="bad")
    assert bad.get_factorization_type() == "bad"
    assert torch.all(bad.X_cov[:, :, :2, 2:] == 0) and torch.all(bad.X_cov[:, :, 2:, :2] == 0)
    with pytest.raises(ValueError):
        TemporalAMEStructuredMFVI(m, factorization="invalid")


def test_naive_init_api(temporal_model):
    from ame_amd import TemporalAMENaiveMFVI
    m = temporal_model
    vi = TemporalAMENaiveMFVI(m, learning_rate=0.01)
    assert vi.lr == 0.01
    eye = torch.eye(m.d) * 0.5
    assert torch.all(vi.X_cov == eye)
    assert vi.predict_forward(n_steps=3).shape == (m.n, 3, m.d)


def test_model_reconstruction_and_states(temporal_model):
    m = temporal_model
    A, M = m.get_states_at_time(2)
    assert torch.equal(A, m.X[:, 2, :2]) and torch.equal(M, m.X[:, 2, 2:])
    with pytest.raises(ValueError):
        m.get_states_at_time(m.T)
    e = m.compute_temporal_reconstruction_error(m.X)
    assert 0.1 < e < 0.4      # = 2 x R's variance 0.1 (ref test is wrong)
    assert m.compute_temporal_reconstruction_error(m.X + 0.5) > e
    assert m.compute_state_prediction_error(m.X) == 0.0


def test_fast_generator_distribution():
    """generate_data_fast: same model, different stream; zero diagonal, swap-consistent."""
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(60, 6, 3, seed=5)
    Y, X = m.generate_data_fast(return_latents=True, seed=9)
    assert Y.shape == (60, 60, 6, 2) and X.shape == (60, 6, 8)
    idx = torch.arange(60)
    assert torch.all(Y[idx, idx] == 0)
    assert torch.equal(Y[:, :, :, 0], Y.transpose(0, 1)[:, :, :, 1])
    e = m.compute_temporal_reconstruction_error(X)
    assert 0.15 < e < 0.25


def _scripted(elbos):
    """Drive BaseVariationalInference.fit with a scripted ELBO sequence."""
    from ame_amd.inference.base import BaseTemporalVariationalInference

    class VI(BaseTemporalVariationalInference):
        def _initialize_variational_params(self):
            self.X_mean = torch.zeros(self.n, self.T, self.d)
            self.k = 0

        def _update_step(self):
            self.k += 1

        def _compute_elbo(self):
            return torch.tensor(elbos[min(self.k, len(elbos)) - 1], dtype=torch.float32)

        def _compute_reconstruction_error(self):
            return 0.5

    class M:
        n, T, d, r, Y = 3, 2, 6, 2, None
    return VI(M(), learning_rate=0.01)


def test_fit_loop_semantics(capsys):
    """base.py:127-208: 3 consecutive sub-tolerance changes -> converged; printing."""
    vi = _scripted([-100.0, -50.0, -49.999, -49.998, -49.997, -49.996, -10.0])
    h = vi.fit(max_iter=10, tolerance=1e-3, verbose=True, check_every=1)
    assert len(h["elbo"]) == 5 and h is vi.history
    out = capsys.readouterr().out
    assert "Starting VI optimization..." in out and "=" * 60 in out
    assert "Iter    0 | ELBO:    -100.00 | MSE: 0.500000" in out
    assert "Converged at iteration 4" in out
    vi2 = _scripted([-100.0, -90.0, -80.0])
    vi2.fit(max_iter=3, tolerance=1e-6, verbose=True)
    assert "Reached maximum iterations without convergence" in capsys.readouterr().out
    assert isinstance(vi2.get_elbo_history()[0], torch.Tensor)
    assert vi2.get_reconstruction_history() == [0.5, 0.5, 0.5]
    # history accumulates across fit() calls (base.py:208)
    vi2.fit(max_iter=2, tolerance=0.0, verbose=False)
    assert len(vi2.history["elbo"]) == 5


def test_assemble_matches_oracle_formula():
    """engine.assemble (host ELBO assembly from the 8 device sums) vs oracle."""
    import ame_oracle as O
    from ame_amd.engine import Constants, assemble
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    m = TemporalAMEModel(12, 4, 2, seed=3)
    m.generate_data()
    vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=0.5)
    Y = m.Y.numpy().astype(np.float64)
    Xm = vi.X_mean.numpy().astype(np.float64)
    Xc = vi.X_cov.numpy().astype(np.float64)
    P = {k: getattr(m, k).numpy().astype(np.float64) for k in ("R", "R_inv", "Sigma", "Psi",
                                                               "Phi", "Q")}
    sums = _oracle_sums(O, Y, Xm, Xc, P, m.n, m.T, m.d)
    for variant in ("good", "naive"):
        t = assemble(sums, m.n, m.T, m.d, variant, Constants(m))
        ref = O.elbo_split(Y, Xm, Xc, P, variant)
        assert np.allclose([t["loglik"], t["prior0"], t["trans"], t["entropy"]], ref,
                           rtol=1e-12, atol=1e-9)
        assert abs(t["recon"] - O.recon_error(Y, Xm)) < 1e-12


def _oracle_sums(O, Y, Xm, Xc, P, n, T, d, t_lo=0, prev=None):
    """The 8 device sums (include/ame_amd.h, ame_elbo) computed by numpy."""
    r = (d - 2) // 2
    Ri = P["R_inv"]
    S0i = np.linalg.inv(O.sigma0(P["Sigma"], P["Psi"]))
    Qi = np.linalg.inv(P["Q"])
    iu, ju = np.triu_indices(n, 1)
    off = ~np.eye(n, dtype=bool)
    s = np.zeros(8)
    TL = Xm.shape[1]
    for tl in range(TL):
        mu = O.compute_mean(Xm[:, tl], r)
        res = Y[iu, ju, tl] - mu[iu, ju]
        s[0] += np.einsum("pa,ab,pb->", res, Ri, res)
        s[7] += ((Y[:, :, tl] - mu) ** 2)[off].sum()
        tg = t_lo + tl
        for i in range(n):
            S = Xc[i, tl]
            s[1] += np.trace(S)
            s[6] += np.linalg.slogdet(S)[1]
            if tg == 0:
                s[2] += Xm[i, tl] @ S0i @ Xm[i, tl]
                s[3] += np.trace(S0i @ S)
            else:
                pm = Xm[i, tl - 1] if tl > 0 else prev[i]
                e = Xm[i, tl] - P["Phi"] @ pm
                s[4] += e @ Qi @ e
                s[5] += np.trace(Qi @ S)
    return s
