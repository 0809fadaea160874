"""BASELINE config 2 (n=256, T=64, latent_dim=8, lr=0.01) against the REFERENCE
itself: tests/golden/c2_reference.npz was written by
tests/golden/make_golden_c2.py, which ran Alfieriek/Python-Temporal-AME-SVI's own
TemporalAMEModel.generate_data and fit() (fp32, and fp64 with the default dtype
switched) for good / bad / naive.

Y (33.5 MB) is not committed: ame_amd's reference-stream generator
(TemporalAMEModel.generate_data) rebuilds it here and its SHA-256 must equal
the reference's.  The initial state's digests must match too (the same RNG
stream, structured_mf.py:74-113 / naive_mf.py:71-87).  Then two fit()
iterations on the GPU, one per call, against the reference's trajectories:

* ELBO and MSE after each iteration within 5e-6 relative of the fp64
  reference, and within the reference's own fp32 error (|fp32 - fp64|) plus
  5e-6 of its fp32 run;
* sampled X_mean rows (12 nodes, all t) within 5e-6 * max(1, |mu|) of the fp64
  reference, or no further from it than the reference's fp32 run is;
* sampled X_cov blocks within 1e-6 * max(1, |S|);
* the ELBO split (loglik, prior0, trans, entropy) within 5e-6 of |ELBO|.

Reference call sites: temporal_ame.py:147-220, structured_mf.py:58-338,
naive_mf.py:29-396, base.py:127-208.
"""
import numpy as np
import pytest

from test_reference_c2 import _sha, c2  # noqa: F401  (module fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("method", ["good", "bad", "naive"])
def test_config2_against_reference(method, c2, gpu_device):
    z, m, ysha, _ = c2
    if ysha != str(z["Y_sha256"]):
        pytest.fail("reference-stream Y differs from the reference's (see test above)")
    from ame_amd import TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    lr = float(z["lr"])
    if method == "naive":
        vi = TemporalAMENaiveMFVI(m, learning_rate=lr, device=gpu_device)
    else:
        vi = TemporalAMEStructuredMFVI(m, factorization=method, learning_rate=lr, device=gpu_device)
    f32, f64 = f"{method}_f32__", f"{method}_f64__"
    assert _sha(vi.X_mean.numpy()) == str(z[f32 + "init_mean_sha256"])
    assert _sha(vi.X_cov.numpy()) == str(z[f32 + "init_cov_sha256"])
    nodes, cov_it = z["nodes"], z["cov_it"]
    for it in (1, 2):
        vi.fit(max_iter=1, tolerance=0.0, verbose=False)
        ref64, ref32 = z[f64 + f"mean_rows_{it}"], z[f32 + f"mean_rows_{it}"]
        got = vi.X_mean.numpy()[nodes].astype(np.float64)
        fp32_err = np.abs(ref32 - ref64).max()
        err = np.abs(got - ref64).max()
        assert err <= max(5e-6 * max(1.0, np.abs(ref64).max()), fp32_err), (it, err, fp32_err)
        cref = z[f64 + f"cov_blocks_{it}"]
        cgot = np.stack([vi.X_cov.numpy()[i, t] for i, t in cov_it]).astype(np.float64)
        cerr = np.abs(cgot - cref).max()
        assert cerr <= 1e-6 * max(1.0, np.abs(cref).max()), (it, cerr)
        sp = vi.elbo_terms()
        split = np.array([sp["loglik"], sp["prior0"], sp["trans"], sp["entropy"]])
        sref = z[f64 + "elbo_split"][it - 1]
        assert np.all(np.abs(split - sref) <= 5e-6 * abs(sp["elbo"])), (it, split, sref)
    e = np.array([float(x) for x in vi.history["elbo"]])
    rec = np.array(vi.history["reconstruction_error"])
    e64, e32 = z[f64 + "elbo"], z[f32 + "elbo"]
    r64, r32 = z[f64 + "recon"], z[f32 + "recon"]
    assert np.all(np.abs(e - e64) <= 5e-6 * np.abs(e64)), (e, e64)
    assert np.all(np.abs(rec - r64) <= 5e-6 * np.abs(r64)), (rec, r64)
    # the reference's own fp32 run is within its fp32 error of ours
    assert np.all(np.abs(e - e32) <= np.abs(e32 - e64) + 5e-6 * np.abs(e32)), (e, e32)
    assert np.all(np.abs(rec - r32) <= np.abs(r32 - r64) + 5e-6 * np.abs(r32)), (rec, r32)
