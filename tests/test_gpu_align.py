"""GPU: post-fit alignment kernels (ame_align_cross / ame_align_apply, through
the C-ABI) against the reference's outputs (golden fixtures) and the fp64
oracle; the timing harness and method comparison on a three-way run.

Tolerance: rows within 2e-5 * max(1, |x|) of the reference (fp32) / oracle;
errors and correlations 1e-5 relative.  Row sign decisions are exact except on
ties, which the random inputs here do not produce."""
import numpy as np
import pytest
import torch

import ame_oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag", ["c1", "mid", "wide"])
def test_align_vs_reference(tag, gpu_device):
    from ame_amd.utils import (align_temporal_states, compute_alignment_error,
                               compute_correlation_after_alignment)
    z = golden(f"{tag}_align.npz")
    r = int(z["r"])
    Xt = torch.from_numpy(z["X_true"])
    tol = 2e-5 * max(1.0, float(Xt.abs().max()))
    for name in [k[:-4] for k in z.files if k.endswith("_est")]:
        Xe = torch.from_numpy(z[f"{name}_est"])
        each = align_temporal_states(Xe, Xt, r)
        assert each.device == Xe.device and each.dtype == torch.float32
        assert np.abs(each.numpy() - z[f"{name}_each"]).max() <= tol, name
        glob = align_temporal_states(Xe, Xt, r, align_each_time=False)
        assert np.abs(glob.numpy() - z[f"{name}_global"]).max() <= tol, name
        err, Xa = compute_alignment_error(Xe, Xt, latent_dim=r)
        assert abs(err - z[f"{name}_err"]) <= 1e-5 * z[f"{name}_err"]
        err0, _ = compute_alignment_error(Xe, Xt, latent_dim=r, align=False)
        assert abs(err0 - z[f"{name}_err_noalign"]) <= 1e-5 * z[f"{name}_err_noalign"]
        c = compute_correlation_after_alignment(Xe, Xt, r)
        assert abs(c - z[f"{name}_corr"]) <= 1e-5


def test_align_keeps_fp64_dtype(gpu_device):
    """fp64 inputs come back fp64 (the kernels compute in fp32; the reference
    returns X_est-typed results, alignment.py:275-321)."""
    from ame_amd.utils import align_latent_positions, align_temporal_states
    z = golden("c1_align.npz")
    r = int(z["r"])
    Xt = torch.from_numpy(z["X_true"]).double()
    name = [k[:-4] for k in z.files if k.endswith("_est")][0]
    Xe = torch.from_numpy(z[f"{name}_est"]).double()
    each = align_temporal_states(Xe, Xt, r)
    assert each.dtype == torch.float64 and each.device == Xe.device
    assert np.abs(each.numpy() - z[f"{name}_each"]).max() <= 2e-5 * max(1.0, float(Xt.abs().max()))
    lat = align_latent_positions(Xe[:, 0, 2:], Xt[:, 0, 2:], r)
    assert lat.dtype == torch.float64


@pytest.mark.parametrize("n,T,r", [(1024, 16, 16), (500, 6, 32), (77, 3, 1)])
def test_align_vs_oracle_large(n, T, r, gpu_device):
    """Device-resident inputs at config sizes against the fp64 oracle."""
    from ame_amd.utils import align_temporal_states, compute_alignment_error
    rng = np.random.default_rng(n + r)
    Xt = rng.standard_normal((n, T, 2 + 2 * r)).astype(np.float32)
    Xe = (Xt[:, :, ::-1] * 0.9 + 0.3 * rng.standard_normal(Xt.shape)).astype(np.float32)
    Xe_d = torch.from_numpy(np.ascontiguousarray(Xe)).to(gpu_device)
    Xt_d = torch.from_numpy(Xt).to(gpu_device)
    for each in (True, False):
        got = align_temporal_states(Xe_d, Xt_d, r, align_each_time=each)
        assert got.is_cuda
        ref = O.align_temporal_states(Xe.astype(np.float64), Xt.astype(np.float64), r, each)
        assert np.abs(got.cpu().numpy() - ref).max() <= 2e-5 * max(1.0, np.abs(ref).max()), each
    err, _ = compute_alignment_error(Xe_d, Xt_d, latent_dim=r)
    ref_err, _ = O.compute_alignment_error(Xe.astype(np.float64), Xt.astype(np.float64), r)
    assert abs(err - ref_err) <= 1e-5 * ref_err


def test_static_alignment(gpu_device):
    """(n, d) inputs: the T = 1 path (alignment.py:366-376)."""
    from ame_amd.utils import align_latent_positions, compute_alignment_error
    z = golden("mid_align.npz")
    r = int(z["r"])
    Xe = z["rot_est"][:, 0].astype(np.float64)
    Xt = z["X_true"][:, 0].astype(np.float64)
    err, Xa = compute_alignment_error(torch.from_numpy(Xe).float(), torch.from_numpy(Xt).float(), r)
    ref = O.align_temporal_states(Xe[:, None], Xt[:, None], r, True)[:, 0]
    assert Xa.shape == (Xe.shape[0], Xe.shape[1])
    assert np.abs(Xa.numpy() - ref).max() <= 2e-5 * max(1.0, np.abs(ref).max())
    assert abs(err - float(((ref - Xt) ** 2).mean())) <= 1e-5 * err
    M = align_latent_positions(torch.from_numpy(Xe[:, 2:]).float(), torch.from_numpy(Xt[:, 2:]).float(), r)
    assert np.abs(M.numpy() - O.align_latent_positions(Xe[:, 2:], Xt[:, 2:], r)).max() <= 2e-5 * 4


def test_three_way_with_timing(gpu_device, capsys):
    """demo.py-style three-way run through run_method_with_timing + compare_methods."""
    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    from ame_amd.utils import align_temporal_states, compare_methods, run_method_with_timing
    m = TemporalAMEModel(15, 10, 2, seed=42)
    m.generate_data()
    z = golden("c1_demo100.npz")
    results = {}
    for name, cls, kw in (("Naive MF", TemporalAMENaiveMFVI, {}),
                          ("Good SMF", TemporalAMEStructuredMFVI, {"factorization": "good"}),
                          ("Bad SMF", TemporalAMEStructuredMFVI, {"factorization": "bad"})):
        res = run_method_with_timing(cls, m, name, max_iter=100, verbose=False,
                                     learning_rate=0.01, device=gpu_device, **kw)
        assert res["iterations"] == 100 and res["runtime"] > 0
        assert set(res["kernels_ms"]) >= {"sweep", "cov", "elbo"}
        key = {"Naive MF": "naive", "Good SMF": "good", "Bad SMF": "bad"}[name]
        assert np.abs(res["X_est"].numpy() - z[f"{key}_mean"]).max() < 2e-4
        res["X_est"] = align_temporal_states(res["X_est"], m.X, 2)
        results[name] = res
    compare_methods(results, metric="reconstruction_error", X_true=m.X)
    out = capsys.readouterr().out
    assert "Method Comparison" in out and "Improvement over" in out
