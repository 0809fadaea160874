"""Generate golden fixtures for the SMF / naive-MF VI hot path from the reference.

TEST INFRASTRUCTURE ONLY.  Runs in the build container, where the reference
(Alfieriek/Python-Temporal-AME-SVI) is mounted read-only at /root/reference.
It imports the reference's own classes, runs them on seeded synthetic inputs
and writes plain-data ``.npz`` files (inputs + expected outputs) next to this
script.  Nothing here ships; nothing on the GPU box reads /root/reference.

Usage (from the repo root)::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Reference call sites exercised (file:line under /root/reference):
  * TemporalAMEModel.__init__ / generate_data   src/models/temporal_ame.py:93-220
  * TemporalAMEStructuredMFVI.__init__ / init   src/inference/structured_mf.py:58-113
  * BaseVariationalInference.fit                src/inference/base.py:127-208
  * _compute_expected_log_likelihood etc.       src/inference/structured_mf.py:115-209
  * _compute_observation_terms                  src/inference/structured_mf.py:289-326
  * TemporalAMENaiveMFVI                         src/inference/naive_mf.py:29-396
"""
import os
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

sys.dont_write_bytecode = True
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from src.models import TemporalAMEModel  # noqa: E402
from src.inference import TemporalAMEStructuredMFVI, TemporalAMENaiveMFVI  # noqa: E402


def model_arrays(m):
    return dict(
        Y=m.Y.numpy(), X_true=m.X.numpy(), R=m.R.numpy(), R_inv=m.R_inv.numpy(),
        Sigma=m.Sigma.numpy(), Psi=m.Psi.numpy(), Phi=m.Phi.numpy(), Q=m.Q.numpy(),
        n=np.int64(m.n), T=np.int64(m.T), r=np.int64(m.r), d=np.int64(m.d),
    )


def elbo_split(vi):
    return np.array([
        float(vi._compute_expected_log_likelihood()),
        float(vi._compute_log_prior_initial()),
        float(vi._compute_log_prior_transitions()),
        float(vi._compute_entropy()),
    ], dtype=np.float64)


def make_vi(method, model, lr):
    if method == "naive":
        return TemporalAMENaiveMFVI(model, learning_rate=lr)
    return TemporalAMEStructuredMFVI(model, factorization=method, learning_rate=lr)


def to_f64(model, vi):
    """fp64 oracle mode: every float tensor attribute -> double."""
    for obj in (model, vi):
        for k, v in list(vars(obj).items()):
            if isinstance(v, torch.Tensor) and v.is_floating_point():
                setattr(obj, k, v.double())
    vi.Y = model.Y


def run_trajectory(model, method, lr, iters, snaps, keep_cov_at, f64=False):
    """Run fit() one iteration at a time, capturing state after selected iterations."""
    vi = make_vi(method, model, lr)
    rec = {}
    rec["init_mean"] = vi.X_mean.clone().numpy()
    rec["init_cov"] = vi.X_cov.clone().numpy()
    prev_dtype = torch.get_default_dtype()
    if f64:
        to_f64(model, vi)
        torch.set_default_dtype(torch.float64)
    try:
        splits = []
        for it in range(1, iters + 1):
            vi.fit(max_iter=1, tolerance=0.0, verbose=False)
            splits.append(elbo_split(vi))
            if it in snaps:
                rec[f"mean_{it}"] = vi.X_mean.clone().numpy()
            if it in keep_cov_at:
                rec[f"cov_{it}"] = vi.X_cov.clone().numpy()
        rec["elbo"] = np.array([float(e) for e in vi.history["elbo"]], dtype=np.float64)
        rec["recon"] = np.array(vi.history["reconstruction_error"], dtype=np.float64)
        rec["elbo_split"] = np.stack(splits)
    finally:
        torch.set_default_dtype(prev_dtype)
    return rec


def build_model(n, T, r, seed=42, **kw):
    m = TemporalAMEModel(n_nodes=n, n_time=T, latent_dim=r, seed=seed, **kw)
    m.generate_data(return_latents=True)
    return m


def save(name, arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)/1024:.1f} KiB)")


def gen_config(tag, n, T, r, runs, iters, snaps, keep_cov_at, with_f64):
    """One fixture file per (method, lr); the model arrays are stored once per config."""
    m = build_model(n, T, r, ar_coefficient=0.8, rho_dyadic=0.5)
    save(f"{tag}_model.npz", model_arrays(m))
    for method, lr in runs:
        for f64 in ([False, True] if with_f64 else [False]):
            mm = build_model(n, T, r, ar_coefficient=0.8, rho_dyadic=0.5)  # fresh copy
            rec = run_trajectory(mm, method, lr, iters, snaps, keep_cov_at, f64=f64)
            rec["lr"] = np.float64(lr)
            rec["iters"] = np.int64(iters)
            suffix = "_f64" if f64 else ""
            save(f"{tag}_{method}_lr{lr:g}{suffix}.npz", rec)


def gen_single_step():
    """Observation terms and one node update at config-1 init."""
    m = build_model(15, 10, 2, ar_coefficient=0.8, rho_dyadic=0.5)
    out = {}
    for method in ("good", "bad"):
        vi = TemporalAMEStructuredMFVI(m, factorization=method, learning_rate=1.0)
        Ps, hs, its = [], [], []
        for (i, t) in [(0, 0), (3, 4), (14, 9), (7, 0)]:
            P, h = vi._compute_observation_terms(i, t)
            Ps.append(P.numpy()); hs.append(h.numpy()); its.append((i, t))
        out[f"{method}_obs_P"] = np.stack(Ps)
        out[f"{method}_obs_h"] = np.stack(hs)
        out[f"{method}_obs_it"] = np.array(its, dtype=np.int64)
        out[f"{method}_before_mean"] = vi.X_mean.clone().numpy()
        out[f"{method}_before_cov"] = vi.X_cov.clone().numpy()
        vi._update_node_i(0)
        out[f"{method}_after0_mean"] = vi.X_mean.clone().numpy()
        out[f"{method}_after0_cov"] = vi.X_cov.clone().numpy()
    save("c1_single_step.npz", out)


def gen_demo_trajectory():
    """Config 1 exactly as demo.py (lr=0.01) for 100 iterations: full ELBO/MSE curve."""
    out = {}
    for method in ("good", "bad", "naive"):
        m = build_model(15, 10, 2, ar_coefficient=0.8, rho_dyadic=0.5)
        vi = make_vi(method, m, 0.01)
        h = vi.fit(max_iter=100, verbose=False)
        out[f"{method}_elbo"] = np.array([float(e) for e in h["elbo"]], dtype=np.float64)
        out[f"{method}_recon"] = np.array(h["reconstruction_error"], dtype=np.float64)
        out[f"{method}_mean"] = vi.X_mean.numpy()
    save("c1_demo100.npz", out)


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    # Config 1 = demo.py (n=15, T=10, r=2, seed 42).
    gen_config("c1", 15, 10, 2,
               runs=[("good", 0.01), ("good", 1.0), ("bad", 0.01), ("bad", 1.0),
                     ("naive", 0.01), ("naive", 1.0)],
               iters=5, snaps={1, 2, 5}, keep_cov_at={1, 5}, with_f64=True)
    # Reference test fixture size (tests/conftest.py:34-43): n=10, T=5, r=2.
    gen_config("tfix", 10, 5, 2, runs=[("good", 1.0), ("bad", 1.0), ("naive", 1.0)],
               iters=3, snaps={1, 3}, keep_cov_at={3}, with_f64=False)
    # Mid config (n=40, T=12, r=3): odd r, d=8.
    gen_config("mid", 40, 12, 3, runs=[("good", 0.01), ("good", 1.0), ("bad", 1.0),
                                       ("naive", 0.01)],
               iters=2, snaps={1, 2}, keep_cov_at={2}, with_f64=True)
    gen_single_step()
    gen_demo_trajectory()
