"""Loop-structured CPU restatement of the temporal-AME SMF hot path.

TEST / BASELINE INFRASTRUCTURE ONLY (same rules as ame_oracle.py: only
``tests/`` and ``bench.py``'s ``cpu_baseline`` leg use it, never the product
path).  SURVEY.md §8d(i): the CPU baseline that keeps the reference's cost
model -- one small torch CPU operation sequence per ordered dyad in the update
and per unordered pair in the ELBO, fp32 -- so its time per dyad is what the
reference pays on the same host.  The vectorised ``ame_oracle`` is the *fair*
CPU baseline (§8d(ii)); this one is the *reference-shaped* one.

Follows (Alfieriek/Python-Temporal-AME-SVI):
  update of node i at time t        src/inference/structured_mf.py:240-287
  observation terms, per-j loop     src/inference/structured_mf.py:303-324
  expected log-likelihood, per pair src/inference/structured_mf.py:130-148

Pinned by tests/test_loop_oracle.py against ame_oracle (itself pinned to the
reference's golden fixtures).
"""
from __future__ import annotations

import math

import torch

LOG2PI = math.log(2.0 * math.pi)


def _consts(params, d):
    f = torch.float32
    R_inv = torch.as_tensor(params["R_inv"], dtype=f)
    Phi = torch.as_tensor(params["Phi"], dtype=f)
    Q_inv = torch.linalg.inv(torch.as_tensor(params["Q"], dtype=f))
    S0 = torch.zeros(d, d)
    S0[:2, :2] = torch.as_tensor(params["Sigma"], dtype=f)
    S0[2:, 2:] = torch.as_tensor(params["Psi"], dtype=f)
    return R_inv, Phi, Q_inv, torch.linalg.inv(S0)


def obs_terms_loop(Y, X_mean, R_inv, i, t, r):
    """P_obs, h_obs of node i at time t, one J per other node j (:303-324)."""
    n, _, d = X_mean.shape
    P = torch.zeros(d, d)
    h = torch.zeros(d)
    M = X_mean[:, t, 2:]
    for j in range(n):
        if j == i:
            continue
        J = torch.zeros(2, d)
        J[0, 0] = 1.0
        J[0, 2:2 + r] = M[j, r:]
        J[1, 1] = 1.0
        J[1, 2 + r:] = M[j, :r]
        RJ = R_inv @ J
        P += J.t() @ RJ
        h += J.t() @ (R_inv @ Y[i, j, t])
    return P, h


def update_step_loop(Y, X_mean, X_cov, params, i, t, variant, lr, consts=None):
    """One (node i, time t) step of the sweep, in place (:240-287)."""
    n, T, d = X_mean.shape
    r = (d - 2) // 2
    R_inv, Phi, Q_inv, S0_inv = consts if consts is not None else _consts(params, d)
    P, h = obs_terms_loop(Y, X_mean, R_inv, i, t, r)
    if t == 0:
        P = P + S0_inv
    if t > 0:
        P = P + Q_inv
        h = h + Q_inv @ (Phi @ X_mean[i, t - 1])
    if t < T - 1:
        P = P + Phi.t() @ (Q_inv @ Phi)
        h = h + Phi.t() @ (Q_inv @ X_mean[i, t + 1])
    if variant == "naive":
        mu = torch.linalg.solve(P, h)
        C = torch.diag(1.0 / (torch.diagonal(P) + 1e-8))
    else:
        C = torch.linalg.inv(P)
        if variant == "bad":
            C[:2, 2:] = 0
            C[2:, :2] = 0
        C = (C + C.t()) / 2 + torch.eye(d) * 1e-6
        mu = C @ h
    X_mean[i, t] = lr * mu + (1 - lr) * X_mean[i, t]
    X_cov[i, t] = lr * C + (1 - lr) * X_cov[i, t]


def update_node_loop(Y, X_mean, X_cov, params, i, variant, lr, ts=None):
    consts = _consts(params, X_mean.shape[2])
    for t in (range(X_mean.shape[1]) if ts is None else ts):
        update_step_loop(Y, X_mean, X_cov, params, i, t, variant, lr, consts)


def loglik_pairs_loop(Y, X_mean, X_cov, params, variant, t, pairs=None):
    """Sum over unordered pairs (i<j) at time t of the loglik term (:130-148);
    ``pairs``: optional iterable of (i, j) to evaluate (a sample)."""
    n, T, d = X_mean.shape
    r = (d - 2) // 2
    R_inv = torch.as_tensor(params["R_inv"], dtype=torch.float32)
    logdetR = torch.logdet(torch.as_tensor(params["R"], dtype=torch.float32))
    trRi = torch.trace(R_inv)
    A, M = X_mean[:, t, :2], X_mean[:, t, 2:]
    add = A[:, 0].unsqueeze(1) + A[:, 1].unsqueeze(0)
    mult = M[:, :r] @ M[:, r:].t()
    mu = torch.stack([add + mult, add.t() + mult.t()], dim=-1)
    if pairs is None:
        pairs = ((i, j) for i in range(n) for j in range(i + 1, n))
    tot = torch.zeros(())
    for i, j in pairs:
        res = Y[i, j, t] - mu[i, j]
        q = res @ (R_inv @ res)
        if variant == "naive":
            corr = 0.0
        else:
            corr = 0.1 * (torch.trace(X_cov[i, t]) + torch.trace(X_cov[j, t])) * trRi / d
        tot = tot + (-0.5 * (logdetR + q + corr + 2 * LOG2PI))
    return tot
