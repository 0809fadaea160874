"""Pin the statistics form of the oracle sweep (ame_oracle.sweep_stats) to the
direct restatement (ame_oracle.sweep) and to the reference's own fp64 runs.

sweep_stats is what the GPU tests replay full sweeps with at the BASELINE
shapes (n = 1024 and 4096), where the direct restatement takes minutes per
sweep.  Same node order, same per-step formulas (structured_mf.py:211-287,
naive_mf.py:207-282); P_obs / h_obs come from running sums.
"""
import glob
import os

import numpy as np
import pytest

import ame_oracle as O
from conftest import GOLDEN, golden, golden_params


@pytest.mark.parametrize("n,T,r,method,lr", [
    (12, 5, 2, "good", 0.7), (15, 6, 3, "bad", 1.0), (11, 4, 1, "naive", 0.3),
    (30, 8, 4, "good", 0.01), (9, 1, 2, "good", 0.5), (2, 3, 5, "bad", 0.2),
    (17, 7, 3, "naive", 1.0)])
def test_stats_sweep_equals_direct(n, T, r, method, lr):
    rng = np.random.default_rng(n * 100 + T)
    d = 2 + 2 * r
    P = {k: v.astype(np.float64) for k, v in O.model_params(r).items()}
    Y = rng.standard_normal((n, n, T, 2)).astype(np.float32)   # non-zero diagonal: j != i masked
    Xm = rng.standard_normal((n, T, d)) * 0.3
    Xc = np.tile(np.eye(d) * 0.5, (n, T, 1, 1)) + rng.standard_normal((n, T, d, d)) * 1e-3
    A = (Xm.copy(), Xc.copy())
    B = (Xm.copy(), Xc.copy())
    for _ in range(2):
        O.sweep(Y, A[0], A[1], P, method, lr)
        O.sweep_stats(Y, B[0], B[1], P, method, lr)
    assert np.abs(A[0] - B[0]).max() <= 1e-12 * max(1.0, np.abs(A[0]).max())
    assert np.abs(A[1] - B[1]).max() <= 1e-13 * max(1.0, np.abs(A[1]).max())


def test_stats_sweep_node_prefix():
    """nodes=range(K) replays the first K nodes only (node i needs only the
    pre-sweep state and nodes < i)."""
    rng = np.random.default_rng(3)
    n, T, r = 14, 4, 2
    d = 2 + 2 * r
    P = {k: v.astype(np.float64) for k, v in O.model_params(r).items()}
    Y = rng.standard_normal((n, n, T, 2))
    Xm = rng.standard_normal((n, T, d)) * 0.3
    Xc = np.tile(np.eye(d) * 0.5, (n, T, 1, 1))
    A, B = (Xm.copy(), Xc.copy()), (Xm.copy(), Xc.copy())
    O.sweep_stats(Y, A[0], A[1], P, "good", 0.4, nodes=range(5))
    O.sweep(Y, B[0], B[1], P, "good", 0.4, nodes=range(5))
    assert np.abs(A[0] - B[0]).max() < 1e-13
    assert np.array_equal(A[0][5:], Xm[5:])


@pytest.mark.parametrize("name", sorted(os.path.basename(f) for f in
                                        glob.glob(os.path.join(GOLDEN, "c1_*_lr*_f64.npz"))))
def test_stats_sweep_reference_fp64(name):
    """The reference's own fp64 runs (tests/golden/make_golden.py) at config 1."""
    z = golden(name)
    tag, method = name.split("_")[:2]
    P = golden_params(tag, np.float64)
    Y = golden(f"{tag}_model.npz")["Y"].astype(np.float64)
    Xm = z["init_mean"].astype(np.float64).copy()
    Xc = z["init_cov"].astype(np.float64).copy()
    lr = float(z["lr"])
    for it in range(1, int(z["iters"]) + 1):
        O.sweep_stats(Y, Xm, Xc, P, method, lr)
        if f"mean_{it}" in z:
            assert np.abs(Xm - z[f"mean_{it}"]).max() < 1e-11, it
        if f"cov_{it}" in z:
            assert np.abs(Xc - z[f"cov_{it}"]).max() < 1e-13, it


def test_stats_sweep_reference_config2():
    """BASELINE config 2 (n=256, T=64, r=8): two sweeps from the reference's
    initial state against the reference's fp64 run (c2_reference.npz)."""
    fix = os.path.join(GOLDEN, "c2_reference.npz")
    if not os.path.exists(fix):
        pytest.skip("c2_reference.npz not generated")
    import torch
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    z = np.load(fix)
    m = TemporalAMEModel(int(z["n"]), int(z["T"]), int(z["r"]), ar_coefficient=0.8,
                         rho_dyadic=0.5, seed=42)
    m.generate_data(X=torch.from_numpy(z["X_true"]))
    lr = float(z["lr"])
    vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=lr)
    Xm = vi.X_mean.numpy().astype(np.float64)
    Xc = vi.X_cov.numpy().astype(np.float64)
    params = {k: getattr(m, k).numpy().astype(np.float64)
              for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")}
    Y = m.Y.numpy()
    for _ in range(2):
        O.sweep_stats(Y, Xm, Xc, params, "good", lr)
    assert np.abs(Xm[z["nodes"]] - z["good_f64__mean_rows_2"]).max() < 1e-9
    e = O.elbo(Y.astype(np.float64), Xm, Xc, params, "good")
    assert abs(e - z["good_f64__elbo"][1]) <= 1e-9 * abs(z["good_f64__elbo"][1])


@pytest.mark.parametrize("method", ["good", "bad", "naive"])
def test_elbo_recon_fast_equals_direct(method):
    rng = np.random.default_rng(11)
    n, T, r = 13, 4, 3
    d = 2 + 2 * r
    P = {k: v.astype(np.float64) for k, v in O.model_params(r).items()}
    Y = rng.standard_normal((n, n, T, 2))
    Y = Y + np.swapaxes(Y[..., ::-1], 0, 1)            # swap-consistent, like the model's Y
    Xm = rng.standard_normal((n, T, d)) * 0.3
    A = rng.standard_normal((n, T, d, d)) * 0.05
    Xc = np.eye(d) * 0.5 + A @ np.swapaxes(A, 2, 3)
    split, rec = O.elbo_recon_fast(Y, Xm, Xc, P, method)
    ref = O.elbo_split(Y, Xm, Xc, P, method)
    assert np.allclose(split, ref, rtol=1e-11, atol=1e-9)
    assert abs(rec - O.recon_error(Y, Xm)) <= 1e-12 * rec
