"""Pin the CPU oracle (oracle/ame_oracle.py) to the reference's own outputs.

The golden fixtures were produced by running the reference itself
(tests/golden/make_golden.py).  fp64 fixtures come from the reference run in
float64; the oracle must reproduce them to ~1e-12.  fp32
fixtures come from the reference's default dtype; the oracle's fp32 run differs
only by summation order (<= 3e-5 on the means at n=40, lr=1).
"""
import glob
import os

import numpy as np
import pytest

import ame_oracle as O
from conftest import GOLDEN, golden, golden_params


def _runs(f64):
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "*_lr*.npz"))):
        name = os.path.basename(f)
        if name.endswith("_f64.npz") != f64:
            continue
        out.append(name)
    return out


def _replay(name, dt):
    z = golden(name)
    tag, method = name.split("_")[:2]
    P = golden_params(tag, dt)
    Y = golden(f"{tag}_model.npz")["Y"].astype(dt)
    Xm = z["init_mean"].astype(dt).copy()
    Xc = z["init_cov"].astype(dt).copy()
    lr = float(z["lr"])
    res = []
    for it in range(1, int(z["iters"]) + 1):
        O.sweep(Y, Xm, Xc, P, method, lr)
        sp = O.elbo_split(Y, Xm, Xc, P, method)
        res.append((it, Xm.copy(), Xc.copy(), sp, O.recon_error(Y, Xm)))
    return z, res


@pytest.mark.parametrize("name", [n for n in _runs(True) if not n.startswith("mid")])
def test_oracle_fp64_exact(name):
    z, res = _replay(name, np.float64)
    for it, Xm, Xc, sp, rec in res:
        if f"mean_{it}" in z:
            assert np.abs(Xm - z[f"mean_{it}"]).max() < 1e-12
        if f"cov_{it}" in z:
            assert np.abs(Xc - z[f"cov_{it}"]).max() < 1e-14
        assert abs(sp.sum() - z["elbo"][it - 1]) <= 1e-12 * abs(z["elbo"][it - 1])
        assert np.all(np.abs(sp - z["elbo_split"][it - 1]) <= 1e-9)
        assert abs(rec - z["recon"][it - 1]) <= 1e-12 * z["recon"][it - 1]


@pytest.mark.parametrize("name", [n for n in _runs(False) if n.startswith(("c1", "tfix"))])
def test_oracle_fp32_close(name):
    z, res = _replay(name, np.float32)
    for it, Xm, Xc, sp, rec in res:
        if f"mean_{it}" in z:
            assert np.abs(Xm - z[f"mean_{it}"]).max() < 5e-6
        assert abs(sp.sum() - z["elbo"][it - 1]) <= 5e-6 * abs(z["elbo"][it - 1])


def test_oracle_mid_fp64_first_iteration():
    """n=40, T=12, r=3 (odd r) — first iteration only, to keep the CPU suite fast."""
    name = "mid_good_lr1_f64.npz"
    z = golden(name)
    P = golden_params("mid")
    Y = golden("mid_model.npz")["Y"].astype(np.float64)
    Xm = z["init_mean"].astype(np.float64).copy()
    Xc = z["init_cov"].astype(np.float64).copy()
    O.sweep(Y, Xm, Xc, P, "good", 1.0)
    assert np.abs(Xm - z["mean_1"]).max() < 1e-11
    e = O.elbo(Y, Xm, Xc, P, "good")
    assert abs(e - z["elbo"][0]) <= 1e-12 * abs(z["elbo"][0])


def test_observation_terms_single_step():
    """_compute_observation_terms(i,t) at init (structured_mf.py:289-326)."""
    z = golden("c1_single_step.npz")
    P = golden_params("c1", np.float32)
    Y = golden("c1_model.npz")["Y"]
    for method in ("good", "bad"):
        Xm = z[f"{method}_before_mean"]
        for (i, t), Pr, hr in zip(z[f"{method}_obs_it"], z[f"{method}_obs_P"],
                                  z[f"{method}_obs_h"]):
            Po, ho = O.observation_terms(Y, Xm, P["R_inv"], int(i), int(t))
            assert np.allclose(Po, Pr, rtol=2e-6, atol=2e-5)
            assert np.allclose(ho, hr, rtol=2e-6, atol=2e-5)
        Xm2 = Xm.copy()
        Xc2 = z[f"{method}_before_cov"].copy()
        O.update_node(Y, Xm2, Xc2, P, 0, method, 1.0)
        assert np.abs(Xm2 - z[f"{method}_after0_mean"]).max() < 5e-6
        assert np.abs(Xc2 - z[f"{method}_after0_cov"]).max() < 1e-7


def test_model_params_match_reference():
    for tag, r in (("c1", 2), ("mid", 3)):
        m = golden(f"{tag}_model.npz")
        p = O.model_params(r)
        for k in ("R", "Sigma", "Psi", "Phi", "Q"):
            assert np.array_equal(p[k], m[k]), (tag, k)
