"""CPU oracle for the temporal-AME structured/naive mean-field VI hot path.

TEST INFRASTRUCTURE ONLY.  This module is a plain-numpy restatement of the
reference algorithm (Alfieriek/Python-Temporal-AME-SVI, ``src/inference``).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker / CPU baseline.  The product path
(``ame_amd``) never imports it and fails loudly without its HIP library.

Parity pin: every function below is checked against golden fixtures produced by
running the reference itself (``tests/golden/make_golden.py`` imports
/root/reference in the build container and writes ``tests/golden/*.npz``).
See ``tests/test_oracle_golden.py``.

Layout follows the reference: ``X_mean (n, T, d)``, ``X_cov (n, T, d, d)``,
``Y (n, n, T, 2)``, state ``x = [a, b, U(r), V(r)]``, ``d = 2 + 2r``
(src/models/temporal_ame.py:114-120).

The arithmetic dtype is the dtype of the arrays passed in (float32 mirrors the
reference's default dtype; float64 is the "fp64 oracle" of SURVEY App. C).
"""
from __future__ import annotations

import math

import numpy as np

LOG2PI = math.log(2.0 * math.pi)


# ----------------------------------------------------------------------------
# model constants (src/models/base.py:123-196, static_ame.py:96-127,
# temporal_ame.py:129-145)
# ----------------------------------------------------------------------------
def cov_matrix(dim, correlation, variance, dtype=np.float32):
    """BaseAMEModel._generate_covariance_matrix (src/models/base.py:123-153)."""
    c = np.full((dim, dim), correlation * variance, dtype=dtype)
    np.fill_diagonal(c, variance)
    return c


def model_params(r, ar=0.8, rho_add=0.5, rho_mult=0.3, rho_dyadic=0.5,
                 process_noise_scale=0.1, dtype=np.float32):
    """R, R_inv, Sigma, Psi, Phi, Q exactly as the reference model builds them."""
    d = 2 + 2 * r
    # R overrides the base-class R (static_ame.py:96-101): var 0.1, corr rho_dyadic.
    R = cov_matrix(2, rho_dyadic, 0.1, dtype)
    R_inv = np.linalg.inv(R.astype(np.float64)).astype(dtype)
    Sigma = cov_matrix(2, rho_add, 1.0, dtype)                     # static_ame.py:111-118
    Psi = np.zeros((2 * r, 2 * r), dtype)                           # static_ame.py:120-127
    Psi[:r, :r] = cov_matrix(r, rho_mult, 1.0, dtype)
    Psi[r:, r:] = cov_matrix(r, rho_mult, 1.0, dtype)
    Phi = np.eye(d, dtype=dtype) * dtype(ar)                          # temporal_ame.py:132
    S0 = sigma0(Sigma, Psi)
    Q = (S0 * dtype(1 - ar ** 2)) * dtype(process_noise_scale)     # temporal_ame.py:144-145
    return dict(R=R, R_inv=R_inv, Sigma=Sigma, Psi=Psi, Phi=Phi, Q=Q)


def sigma0(Sigma, Psi):
    """blockdiag(Sigma, Psi) as built in structured_mf.py:234-236."""
    d = 2 + Psi.shape[0]
    S0 = np.zeros((d, d), dtype=Sigma.dtype)
    S0[:2, :2] = Sigma
    S0[2:, 2:] = Psi
    return S0


def _inv(a):
    return np.linalg.inv(a)


def _logdet(a):
    """torch.logdet semantics: nan for negative determinant, -inf for zero."""
    sign, ld = np.linalg.slogdet(a.astype(np.float64))
    if sign < 0:
        return float("nan")
    if sign == 0:
        return float("-inf")
    return float(ld)


# ----------------------------------------------------------------------------
# observation terms (structured_mf.py:289-326 / naive_mf.py:284-376)
# ----------------------------------------------------------------------------
def observation_terms(Y, X_mean, R_inv, i, t):
    """P_obs = sum_{j!=i} J^T R^-1 J, h_obs = sum_{j!=i} J^T R^-1 y_ij.

    J_j = [[1, 0, V_j, 0], [0, 1, 0, U_j]] (structured_mf.py:309-320).  Summed over
    all j != i with the *current* means (new for j < i inside a sweep).
    """
    n, T, d = X_mean.shape
    r = (d - 2) // 2
    dt = X_mean.dtype
    mask = np.ones(n, dtype=bool)
    mask[i] = False
    M = X_mean[mask, t, 2:]
    U, V = M[:, :r], M[:, r:]
    m = M.shape[0]
    E0 = np.zeros((m, d), dt)
    E1 = np.zeros((m, d), dt)
    E0[:, 0] = 1
    E0[:, 2:2 + r] = V
    E1[:, 1] = 1
    E1[:, 2 + r:] = U
    p, q, s = R_inv[0, 0], R_inv[0, 1], R_inv[1, 1]
    q2 = R_inv[1, 0]
    P = p * (E0.T @ E0) + q * (E0.T @ E1) + q2 * (E1.T @ E0) + s * (E1.T @ E1)
    y = Y[i, mask, t, :]                     # (m, 2)
    z = y @ R_inv.T                          # z_j = R_inv @ y_ij
    h = E0.T @ z[:, 0] + E1.T @ z[:, 1]
    return P.astype(dt), h.astype(dt)


def prior_terms(params, T, dtype):
    Q_inv = _inv(params["Q"]).astype(dtype)
    S0_inv = _inv(sigma0(params["Sigma"], params["Psi"])).astype(dtype)
    Phi = params["Phi"]
    PtQiP = (Phi.T @ (Q_inv @ Phi)).astype(dtype)
    return Q_inv, S0_inv, PtQiP


# ----------------------------------------------------------------------------
# the sweep (structured_mf.py:211-287, naive_mf.py:193-282)
# ----------------------------------------------------------------------------
def update_node(Y, X_mean, X_cov, params, i, variant, lr, consts=None):
    """One node's forward sweep over t, in place.  variant in {good, bad, naive}."""
    n, T, d = X_mean.shape
    dt = X_mean.dtype
    Q_inv, S0_inv, PtQiP = consts if consts is not None else prior_terms(params, T, dt)
    Phi = params["Phi"]
    R_inv = params["R_inv"]
    eye = np.eye(d, dtype=dt)
    for t in range(T):
        P_obs, h_obs = observation_terms(Y, X_mean, R_inv, i, t)
        P = P_obs.copy()
        h = h_obs.copy()
        if t == 0:
            P = P + S0_inv
        if t > 0:
            P = P + Q_inv
            h = h + Q_inv @ (Phi @ X_mean[i, t - 1])
        if t < T - 1:
            P = P + PtQiP
            h = h + Phi.T @ (Q_inv @ X_mean[i, t + 1])
        if variant == "naive":
            mu = np.linalg.solve(P, h)
            C = np.diag(dt.type(1.0) / (np.diag(P) + dt.type(1e-8))).astype(dt)
        else:
            C = _inv(P)
            if variant == "bad":
                C[:2, 2:] = 0
                C[2:, :2] = 0
            C = (C + C.T) / dt.type(2)
            C = C + eye * dt.type(1e-6)
            mu = C @ h
        X_mean[i, t] = dt.type(lr) * mu + dt.type(1 - lr) * X_mean[i, t]
        X_cov[i, t] = dt.type(lr) * C + dt.type(1 - lr) * X_cov[i, t]


def update_step(Y, X_mean, X_cov, params, i, t, variant, lr, consts, T_total=None, t_off=0):
    """One (node i, local slice t) step of update_node, for time-sharded replays:
    X_mean holds local slices plus halo slots; global time = t + t_off."""
    n, TL, d = X_mean.shape
    T = TL if T_total is None else T_total
    tg = t + t_off
    dt = X_mean.dtype
    Q_inv, S0_inv, PtQiP = consts
    Phi = params["Phi"]
    P, h = observation_terms(Y, X_mean, params["R_inv"], i, t)
    if tg == 0:
        P = P + S0_inv
    if tg > 0:
        P = P + Q_inv
        h = h + Q_inv @ (Phi @ X_mean[i, t - 1])
    if tg < T - 1:
        P = P + PtQiP
        h = h + Phi.T @ (Q_inv @ X_mean[i, t + 1])
    if variant == "naive":
        mu = np.linalg.solve(P, h)
        C = np.diag(dt.type(1.0) / (np.diag(P) + dt.type(1e-8))).astype(dt)
    else:
        C = _inv(P)
        if variant == "bad":
            C[:2, 2:] = 0
            C[2:, :2] = 0
        C = (C + C.T) / dt.type(2) + np.eye(d, dtype=dt) * dt.type(1e-6)
        mu = C @ h
    X_mean[i, t] = dt.type(lr) * mu + dt.type(1 - lr) * X_mean[i, t]
    X_cov[i, t] = dt.type(lr) * C + dt.type(1 - lr) * X_cov[i, t]


def sweep(Y, X_mean, X_cov, params, variant, lr, nodes=None):
    """_update_step: sequential Gauss-Seidel over nodes (structured_mf.py:217-218)."""
    n, T, d = X_mean.shape
    consts = prior_terms(params, T, X_mean.dtype)
    for i in (range(n) if nodes is None else nodes):
        update_node(Y, X_mean, X_cov, params, i, variant, lr, consts)


# ----------------------------------------------------------------------------
# the same sweep from running sufficient statistics, for
# parity at the BASELINE shapes
# ----------------------------------------------------------------------------
def _slice_stats(M, r):
    """Per-slice sums over nodes of (U, V) terms: M is (T, n, 2r) current (U, V).
    Returns [count, sU, sV, S_UU, S_VV, S_VU] with S_VU = sum_j V_j U_j^T."""
    U, V = M[:, :, :r], M[:, :, r:]
    Ut, Vt = np.swapaxes(U, 1, 2), np.swapaxes(V, 1, 2)
    return [np.full(M.shape[0], float(M.shape[1]), dtype=M.dtype), U.sum(1), V.sum(1),
            np.matmul(Ut, U), np.matmul(Vt, V), np.matmul(Vt, U)]


def _p_obs(st, R_inv, r):
    """P_obs of structured_mf.py:303-324 from the statistics (App. A): with
    e0 = [1, 0, V, 0], e1 = [0, 1, 0, U],
    P = p e0e0^T + q e0e1^T + q' e1e0^T + s e1e1^T summed over the nodes in st."""
    m, sU, sV, SUU, SVV, SVU = st
    T = m.shape[0]
    d = 2 + 2 * r
    p, q, q2, s = R_inv[0, 0], R_inv[0, 1], R_inv[1, 0], R_inv[1, 1]
    A, B, Ub, Vb = 0, 1, slice(2, 2 + r), slice(2 + r, d)
    P = np.zeros((T, d, d), dtype=sU.dtype)
    P[:, A, A] = p * m
    P[:, A, Ub] = p * sV
    P[:, Ub, A] = p * sV
    P[:, Ub, Ub] = p * SVV
    P[:, A, B] = q * m
    P[:, A, Vb] = q * sU
    P[:, Ub, B] = q * sV
    P[:, Ub, Vb] = q * SVU
    P[:, B, A] += q2 * m
    P[:, Vb, A] = q2 * sU
    P[:, B, Ub] += q2 * sV
    P[:, Vb, Ub] = q2 * np.swapaxes(SVU, 1, 2)
    P[:, B, B] = s * m
    P[:, B, Vb] += s * sU
    P[:, Vb, B] = s * sU
    P[:, Vb, Vb] = s * SUU
    return P


def sweep_stats(Y, X_mean, X_cov, params, variant, lr, nodes=None):
    """_update_step (structured_mf.py:211-287, naive_mf.py:207-282) in fp64, in
    place, vectorised over time: the same Gauss-Seidel node order and the same
    per-step formulas as :func:`update_node`, but P_obs / h_obs come from
    per-slice running sums of the other nodes' (U, V) and
    everything that does not depend on mu_{i,t-1}^new is batched over t (P,
    its inverse, the right AR term); only mu_{i,t} = C_t (h_t + Q^-1 Phi
    mu_{i,t-1}) runs as a loop.  Pinned to :func:`sweep` in
    tests/test_oracle_fast.py; used where the direct restatement is too slow
    (full sweeps at n = 1024-4096).  The arithmetic dtype is X_mean's: fp64 is
    the parity oracle; fp32 (the reference's dtype) only times the CPU baseline
    of bench.py."""
    n, T, d = X_mean.shape
    r = (d - 2) // 2
    dt = X_mean.dtype
    assert dt in (np.float64, np.float32) and X_cov.dtype == dt
    R_inv = params["R_inv"].astype(dt)
    Q_inv, S0_inv, PtQiP = prior_terms({k: v.astype(dt) for k, v in params.items()}, T, dt)
    Phi = params["Phi"].astype(dt)
    QiPhi = Q_inv @ Phi
    PhiTQi = Phi.T @ Q_inv
    eye = np.eye(d, dtype=dt)
    M = np.ascontiguousarray(np.swapaxes(X_mean[:, :, 2:], 0, 1))      # (T, n, 2r) current
    st = _slice_stats(M, r)
    for i in (range(n) if nodes is None else nodes):
        own = M[:, i, :]                                                 # (T, 2r) old
        Uo, Vo = own[:, :r], own[:, r:]
        ex = [st[0] - 1.0, st[1] - Uo, st[2] - Vo,
              st[3] - np.einsum("ta,tb->tab", Uo, Uo), st[4] - np.einsum("ta,tb->tab", Vo, Vo),
              st[5] - np.einsum("ta,tb->tab", Vo, Uo)]
        P = _p_obs(ex, R_inv, r)
        yi = np.asarray(Y[i], dtype=dt).transpose(1, 2, 0)             # (T, 2, n)
        z = np.matmul(R_inv, yi)                                        # z_ij = R^-1 y_ij
        z[:, :, i] = 0.0                                                # j != i
        zM = np.matmul(z, M)                                            # (T, 2, 2r)
        h = np.empty((T, d), dtype=dt)
        h[:, :2] = z.sum(2)
        h[:, 2:2 + r] = zM[:, 0, r:]                                    # sum z0 V_j
        h[:, 2 + r:] = zM[:, 1, :r]                                     # sum z1 U_j
        P[0] += S0_inv
        P[1:] += Q_inv
        P[:-1] += PtQiP
        if T > 1:
            h[:-1] += X_mean[i, 1:] @ PhiTQi.T                          # old mu_{i,t+1}
        Pinv = np.linalg.inv(P)
        if variant == "naive":
            C = np.zeros_like(P)
            idx = np.arange(d)
            C[:, idx, idx] = dt.type(1.0) / (P[:, idx, idx] + dt.type(1e-8))
            G = Pinv
        else:
            C = Pinv.copy()
            if variant == "bad":
                C[:, :2, 2:] = 0.0
                C[:, 2:, :2] = 0.0
            C = (C + np.swapaxes(C, 1, 2)) / dt.type(2) + eye * dt.type(1e-6)
            G = C
        lr_, om_ = dt.type(lr), dt.type(1.0 - lr)
        for t in range(T):
            ht = h[t] + (QiPhi @ X_mean[i, t - 1] if t > 0 else dt.type(0))
            X_mean[i, t] = lr_ * (G[t] @ ht) + om_ * X_mean[i, t]
        X_cov[i] = lr_ * C + om_ * X_cov[i]
        new = X_mean[i, :, 2:]
        Un, Vn = new[:, :r], new[:, r:]
        st = [st[0], ex[1] + Un, ex[2] + Vn, ex[3] + np.einsum("ta,tb->tab", Un, Un),
              ex[4] + np.einsum("ta,tb->tab", Vn, Vn), ex[5] + np.einsum("ta,tb->tab", Vn, Un)]
        M[:, i, :] = new


# ----------------------------------------------------------------------------
# ELBO (structured_mf.py:115-209; naive_mf.py:89-191) and recon
# (temporal_ame.py:255-291)
# ----------------------------------------------------------------------------
def compute_mean(X_t, r):
    """StaticAMEModel.compute_mean (static_ame.py:189-238) for one time slice."""
    a, b = X_t[:, 0], X_t[:, 1]
    U, V = X_t[:, 2:2 + r], X_t[:, 2 + r:]
    add = a[:, None] + b[None, :]
    mult = U @ V.T
    mu = np.empty(add.shape + (2,), dtype=X_t.dtype)
    mu[:, :, 0] = add + mult
    mu[:, :, 1] = add.T + mult.T
    return mu


def expected_loglik(Y, X_mean, X_cov, params, variant, ts=None):
    n, T, d = X_mean.shape
    r = (d - 2) // 2
    R_inv = params["R_inv"].astype(np.float64)
    logdetR = _logdet(params["R"])
    trRi = float(np.trace(R_inv))
    iu, ju = np.triu_indices(n, k=1)
    total = 0.0
    for t in (range(T) if ts is None else ts):
        mu = compute_mean(X_mean[:, t].astype(np.float64), r)
        res = Y[iu, ju, t, :].astype(np.float64) - mu[iu, ju]
        quad = np.einsum("pa,ab,pb->p", res, R_inv, res)
        if variant == "naive":
            corr = 0.0
        else:
            tr = np.trace(X_cov[:, t].astype(np.float64), axis1=1, axis2=2)
            corr = 0.1 * (tr[iu] + tr[ju]) * trRi / d
        total += float(np.sum(-0.5 * (logdetR + quad + corr + 2 * LOG2PI)))
    return total


def log_prior_initial(X_mean, X_cov, params):
    n, T, d = X_mean.shape
    S0 = sigma0(params["Sigma"], params["Psi"]).astype(np.float64)
    S0i = np.linalg.inv(S0)
    ld = _logdet(S0)
    mu0 = X_mean[:, 0].astype(np.float64)
    quad = np.einsum("na,ab,nb->n", mu0, S0i, mu0)
    tr = np.einsum("ab,nba->n", S0i, X_cov[:, 0].astype(np.float64))
    return float(np.sum(-0.5 * (ld + quad + tr + d * LOG2PI)))


def log_prior_transitions(X_mean, X_cov, params):
    n, T, d = X_mean.shape
    if T < 2:
        return 0.0
    Q = params["Q"].astype(np.float64)
    Qi = np.linalg.inv(Q)
    ld = _logdet(Q)
    Phi = params["Phi"].astype(np.float64)
    Xm = X_mean.astype(np.float64)
    res = Xm[:, 1:] - np.einsum("ab,ntb->nta", Phi, Xm[:, :-1])
    quad = np.einsum("nta,ab,ntb->nt", res, Qi, res)
    tr = np.einsum("ab,ntba->nt", Qi, X_cov[:, 1:].astype(np.float64))
    return float(np.sum(-0.5 * (ld + quad + tr + d * LOG2PI)))


def entropy(X_cov):
    n, T, d, _ = X_cov.shape
    tot = 0.0
    for i in range(n):
        for t in range(T):
            tot += 0.5 * (d * (1 + LOG2PI) + _logdet(X_cov[i, t]))
    return tot


def elbo_split(Y, X_mean, X_cov, params, variant):
    return np.array([
        expected_loglik(Y, X_mean, X_cov, params, variant),
        log_prior_initial(X_mean, X_cov, params),
        log_prior_transitions(X_mean, X_cov, params),
        entropy(X_cov),
    ])


def elbo(Y, X_mean, X_cov, params, variant):
    return float(np.sum(elbo_split(Y, X_mean, X_cov, params, variant)))


def recon_error(Y, X_mean):
    """compute_temporal_reconstruction_error (temporal_ame.py:255-291)."""
    n, T, d = X_mean.shape
    r = (d - 2) // 2
    off = ~np.eye(n, dtype=bool)
    tot = 0.0
    for t in range(T):
        mu = compute_mean(X_mean[:, t].astype(np.float64), r)
        e = (Y[:, :, t].astype(np.float64) - mu) ** 2
        tot += float(e[off].sum())
    return tot / (n * (n - 1) * T)


def elbo_recon_fast(Y, X_mean, X_cov, params, variant, dtype=np.float64):
    """elbo_split + recon_error of the same state, vectorised per slice in fp64
    (whole n x n residual matrices instead of index gathers; the entropy's
    log-determinants batched).  Same formulas as above (structured_mf.py:124-209,
    naive_mf.py:114-191, temporal_ame.py:255-291); pinned to them in
    tests/test_oracle_fast.py.  Returns (split[4], recon).  `dtype` is the
    elementwise arithmetic type (fp64: the parity oracle; fp32: bench.py's CPU
    baseline in the reference's dtype); the sums are Python floats either way."""
    dt = np.dtype(dtype)
    n, T, d = X_mean.shape
    r = (d - 2) // 2
    R_inv = params["R_inv"].astype(dt)
    p, q, q2, s = R_inv[0, 0], R_inv[0, 1], R_inv[1, 0], R_inv[1, 1]
    logdetR = _logdet(params["R"])
    trRi = float(np.trace(R_inv))
    upper = np.triu(np.ones((n, n), dtype=bool), k=1)
    off = ~np.eye(n, dtype=bool)
    quad_sum = 0.0
    sq_sum = 0.0
    CH = 8                                    # slices per gather: whole cache lines of Y
    for t in range(T):
        if t % CH == 0:
            yc = np.ascontiguousarray(np.moveaxis(Y[:, :, t:t + CH, :], 2, 0), dtype=dt)
        x = X_mean[:, t].astype(dt)
        add = x[:, 0][:, None] + x[:, 1][None, :]
        mult = x[:, 2:2 + r] @ x[:, 2 + r:].T
        m0 = add + mult                       # mean of y_ij[0]
        yt = yc[t % CH]
        e0 = yt[:, :, 0] - m0
        e1 = yt[:, :, 1] - m0.T
        quad = p * e0 * e0 + (q + q2) * e0 * e1 + s * e1 * e1
        quad_sum += float(quad[upper].sum())
        sq_sum += float((e0 * e0 + e1 * e1)[off].sum())
    npairs = T * n * (n - 1) / 2.0
    if variant == "naive":
        corr = 0.0
    else:
        tr = np.trace(X_cov.astype(dt), axis1=2, axis2=3)              # (n, T)
        corr = 0.1 * trRi / d * (n - 1) * float(tr.sum())
    loglik = -0.5 * (npairs * (logdetR + 2 * LOG2PI) + quad_sum + corr)
    sign, ld = np.linalg.slogdet(X_cov.astype(dt).reshape(-1, d, d))
    ld = np.where(sign > 0, ld, np.where(sign == 0, -np.inf, np.nan))
    ent = float(np.sum(0.5 * (d * (1 + LOG2PI) + ld)))
    split = np.array([loglik, log_prior_initial(X_mean, X_cov, params),
                      log_prior_transitions(X_mean, X_cov, params), ent])
    return split, sq_sum / (n * (n - 1) * T)


# ----------------------------------------------------------------------------
# fit (base.py:127-208) without printing
# ----------------------------------------------------------------------------
def fit(Y, X_mean, X_cov, params, variant, lr, max_iter, tolerance=1e-4):
    hist = {"elbo": [], "reconstruction_error": []}
    prev = -np.inf
    patience = 0
    for it in range(max_iter):
        sweep(Y, X_mean, X_cov, params, variant, lr)
        e = elbo(Y, X_mean, X_cov, params, variant)
        hist["elbo"].append(e)
        hist["reconstruction_error"].append(recon_error(Y, X_mean))
        converged = False
        if it > 0:
            rel = abs(e - prev) / (abs(prev) + 1e-8)
            patience = patience + 1 if rel < tolerance else 0
            converged = patience >= 3
        prev = e
        if converged:
            break
    return hist


# ----------------------------------------------------------------------------
# post-fit alignment (src/utils/alignment.py), SURVEY §8f row f4
# ----------------------------------------------------------------------------
def procrustes_alignment(X_est, X_true):
    """alignment.py:75-90: R = U Vt of svd(X_true^T X_est), last row of Vt
    negated when det(R) < 0; returns (X_est R, R)."""
    M = X_true.T @ X_est
    U, _, Vt = np.linalg.svd(M)
    R = U @ Vt
    if np.linalg.det(R) < 0:
        Vt = Vt.copy()
        Vt[-1, :] *= -1
        R = U @ Vt
    return X_est @ R, R


def align_signs_rows(X_est, X_true):
    """alignment.py:137-145 (dim = last): flip row i when -x_i is closer."""
    out = X_est.copy()
    for i in range(X_est.shape[0]):
        if np.linalg.norm(-X_est[i] - X_true[i]) < np.linalg.norm(X_est[i] - X_true[i]):
            out[i] = -out[i]
    return out


def align_latent_positions(M_est, M_true, r):
    """alignment.py:202-221: Procrustes on U and on V separately, then row signs."""
    U, _ = procrustes_alignment(M_est[:, :r], M_true[:, :r])
    V, _ = procrustes_alignment(M_est[:, r:], M_true[:, r:])
    return np.concatenate([align_signs_rows(U, M_true[:, :r]),
                           align_signs_rows(V, M_true[:, r:])], axis=1)


def align_temporal_states(X_est, X_true, r, align_each_time=True):
    """alignment.py:265-321."""
    n, T, d = X_est.shape
    out = X_est.copy()
    if align_each_time:
        for t in range(T):
            out[:, t, :2] = align_signs_rows(X_est[:, t, :2], X_true[:, t, :2])
            out[:, t, 2:] = align_latent_positions(X_est[:, t, 2:], X_true[:, t, 2:], r)
    else:
        _, RM = procrustes_alignment(X_est.mean(axis=1)[:, 2:], X_true.mean(axis=1)[:, 2:])
        for t in range(T):
            out[:, t, :2] = align_signs_rows(X_est[:, t, :2], X_true[:, t, :2])
            out[:, t, 2:] = align_signs_rows(X_est[:, t, 2:] @ RM, X_true[:, t, 2:])
    return out


def compute_alignment_error(X_est, X_true, r, align=True):
    """alignment.py:359-385, temporal (n, T, d) inputs."""
    Xa = align_temporal_states(X_est, X_true, r) if align else X_est
    return float(((Xa.astype(np.float64) - X_true) ** 2).mean()), Xa


def correlation_after_alignment(X_est, X_true, r):
    """alignment.py:414-436."""
    _, Xa = compute_alignment_error(X_est, X_true, r)
    a = Xa.astype(np.float64).ravel()
    b = X_true.astype(np.float64).ravel()
    a = a - a.mean()
    b = b - b.mean()
    den = np.sqrt((a * a).sum() * (b * b).sum())
    return 0.0 if den < 1e-10 else float((a * b).sum() / den)
