"""BASELINE config 2 on the CPU against the reference's own run
(tests/golden/c2_reference.npz, written by tests/golden/make_golden_c2.py):

* ame_amd's reference-stream generator rebuilds the reference's Y and X bit
  for bit (SHA-256; temporal_ame.py:147-220) -- X here, where the fixture was
  made (X's small MKL matvecs round by the host's MKL code path), and Y from the
  reference's X (the fixture's X_true) on any host, which is what the GPU test
  (tests/test_gpu_reference_c2.py) uses on the GPU box;
* the VI classes draw the reference's initial state (digests;
  structured_mf.py:74-113, naive_mf.py:71-87) -- host code, no GPU;
* the fp64 oracle (oracle/ame_oracle.py) follows the reference's fp64
  trajectory over 2 iterations for SMF-good (ELBO / MSE 1e-9 relative,
  sampled means 1e-9).  This pins the oracle at config 2, where
  tests/test_gpu_baseline_shapes.py checks the device against it.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN

FIX = os.path.join(GOLDEN, "c2_reference.npz")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def c2():
    """The config-2 model with Y regenerated from the reference's X."""
    if not os.path.exists(FIX):
        pytest.skip("c2_reference.npz not generated")
    import torch
    from ame_amd import TemporalAMEModel
    z = np.load(FIX)
    n, T, r = int(z["n"]), int(z["T"]), int(z["r"])
    assert _sha(z["X_true"]) == str(z["X_sha256"])
    m = TemporalAMEModel(n, T, r, ar_coefficient=0.8, rho_dyadic=0.5, seed=42)
    Y, X = m.generate_data(return_latents=True, X=torch.from_numpy(z["X_true"]))
    return z, m, _sha(Y.numpy()), _sha(X.numpy())


def test_reference_stream_regenerated(c2):
    z, m, ysha, xsha = c2
    assert xsha == str(z["X_sha256"])
    assert ysha == str(z["Y_sha256"])
    assert np.array_equal(m.Y.numpy()[z["nodes"]][:, :8], z["Y_rows"])


def test_reference_stream_from_seed_alone():
    """Without the reference's X: X (and so Y) from the seed, on this host."""
    if not os.path.exists(FIX):
        pytest.skip("c2_reference.npz not generated")
    from ame_amd import TemporalAMEModel
    z = np.load(FIX)
    m = TemporalAMEModel(int(z["n"]), int(z["T"]), int(z["r"]), ar_coefficient=0.8,
                         rho_dyadic=0.5, seed=42)
    Y, X = m.generate_data(return_latents=True)
    if _sha(X.numpy()) != str(z["X_sha256"]):
        # X comes from small MKL matvecs whose rounding depends on the host's MKL
        # code path (the GPU box's EPYC rounds differently from the fixture
        # host); Y from the reference's X is pinned on every host above
        pytest.skip("seed-only X differs on this host (MKL code path); "
                    "test_reference_stream_regenerated pins Y from the reference's X")
    assert _sha(Y.numpy()) == str(z["Y_sha256"])


@pytest.mark.parametrize("method", ["good", "bad", "naive"])
def test_initial_state_digests(method, c2):
    from ame_amd import TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    z, m, _, _ = c2
    lr = float(z["lr"])
    if method == "naive":
        vi = TemporalAMENaiveMFVI(m, learning_rate=lr)
    else:
        vi = TemporalAMEStructuredMFVI(m, factorization=method, learning_rate=lr)
    assert _sha(vi.X_mean.numpy()) == str(z[f"{method}_f32__init_mean_sha256"])
    assert _sha(vi.X_cov.numpy()) == str(z[f"{method}_f32__init_cov_sha256"])


def test_oracle_follows_reference_fp64(c2):
    import ame_oracle as O
    from ame_amd import TemporalAMEStructuredMFVI
    z, m, _, _ = c2
    lr = float(z["lr"])
    vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=lr)
    Xm = vi.X_mean.numpy().astype(np.float64)
    Xc = vi.X_cov.numpy().astype(np.float64)
    params = {k: getattr(m, k).numpy().astype(np.float64)
              for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")}
    h = O.fit(m.Y.numpy().astype(np.float64), Xm, Xc, params, "good", lr, 2, 0.0)
    assert np.allclose(h["elbo"], z["good_f64__elbo"], rtol=1e-9, atol=0)
    assert np.allclose(h["reconstruction_error"], z["good_f64__recon"], rtol=1e-9, atol=0)
    assert np.abs(Xm[z["nodes"]] - z["good_f64__mean_rows_2"]).max() < 1e-9
