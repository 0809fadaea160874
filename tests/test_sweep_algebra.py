"""CPU model of the HIP sweep kernel's algebra (ame_sweep.hip), checked against
the oracle sweep (oracle/ame_oracle.py), for good / bad / naive.

The kernel never factorises a precision matrix inside the sweep.  Per time
slice t it keeps a fp64 "base" inverse and applies the last step's rank-4
change lazily, through 2x2 algebra on a handful of dot products, so that the
only work between node i-1's new mean and node i's is one matvec plus one
cross-lane reduction.  This file restates exactly that schedule in numpy
(fp64, per slice, node-major like the reference's Gauss-Seidel order) so the
algebra is testable without a GPU.  Notation (structured_mf.py
:211-326):

  F_j    = J_j^T R^-1 J_j,  J_j = [[1,0,V_j,0],[0,1,0,U_j]]  (2 x d)
  P_i    = Pconst(t) + sum_{j != i} F_j (new for j < i, old for j > i)
  K_i    = (P_i - F_{i-1}^new)^-1                 (excludes nodes i-1 and i)
  base   B_i = K_{i-1}  (B_0 = K_0 = P_0^-1; B_1 = K_0)
  K_i    = B_i - L_{i-1} W_{i-1}^T + G_{i-1} X_{i-1}^T     (lazy rank-4)
  W_i    = K_i J_{i-1}^T,  M_i = R + J_{i-1} W_i,  L_i = W_i M_i^-1
  P_i^-1 = K_i - L_i W_i^T
  X_i    = P_i^-1 J_{i+1}^T (old), S_i = R - J_{i+1} X_i, G_i = X_i S_i^-1
  K_{i+1}= P_i^-1 + G_i X_i^T
  mu_i*  = P_i^-1 h_i = u_i + W_i M_i^-1 (y_{i,i-1} - J_{i-1} u_i),  u_i = K_i g_i
where g_i is h_i without node i-1's observation term.  All quantities that
involve K_i are formed from B_i-products (kj = B J^T, v = B g, yv = B Jn^T)
plus the previous step's vectors, so the d x d rank-4 update itself is off
the critical path (the kernel's helper waves do it one step behind).
"""
import numpy as np
import pytest

import ame_oracle as O


def _inv2(m):
    a, b, c, d = m[0, 0], m[0, 1], m[1, 0], m[1, 1]
    idet = 1.0 / (a * d - b * c)
    out = np.array([[d * idet, -b * idet], [-c * idet, a * idet]])
    out[0, 1] = out[1, 0] = 0.5 * (out[0, 1] + out[1, 0])
    return out


def _J(mu, r):
    """J of a node (2 x d) from its mean (only U, V enter)."""
    d = 2 + 2 * r
    J = np.zeros((2, d))
    J[0, 0] = 1.0
    J[1, 1] = 1.0
    J[0, 2:2 + r] = mu[2 + r:]
    J[1, 2 + r:] = mu[2:2 + r]
    return J


def sweep_lazy(Y, Xm, Xc, params, variant, lr):
    """One sweep with the kernel's schedule; Xm, Xc (fp32) updated in place."""
    n, T, d = Xm.shape
    r = (d - 2) // 2
    f32 = np.float32
    Ri = params["R_inv"].astype(np.float64)
    Rm = _inv2(Ri)
    Qi = np.linalg.inv(params["Q"].astype(np.float64))
    Qi = 0.5 * (Qi + Qi.T)
    S0 = O.sigma0(params["Sigma"], params["Psi"]).astype(np.float64)
    S0i = np.linalg.inv(S0)
    S0i = 0.5 * (S0i + S0i.T)
    Phi = params["Phi"].astype(np.float64)
    PtQiP = Phi.T @ Qi @ Phi
    PtQiP = 0.5 * (PtQiP + PtQiP.T)
    QiPhi, PhiTQi = Qi @ Phi, Phi.T @ Qi
    lr32, om32 = f32(lr), f32(1.0 - lr)
    old = Xm.astype(np.float64).copy()          # means at sweep start

    def pconst(t):
        P = S0i.copy() if t == 0 else Qi.copy()
        if t < T - 1:
            P = P + PtQiP
        return P

    def Fsum(t, excl):
        P = np.zeros((d, d))
        for j in range(n):
            if j in excl:
                continue
            Jj = _J(old[j, t], r)
            P += Jj.T @ Ri @ Jj
        return P

    st = []
    for t in range(T):
        P0 = pconst(t) + Fsum(t, {0})
        z = np.zeros((d, 2))
        st.append(dict(B=np.linalg.inv(P0), L=z.copy(), W=z.copy(), G=z.copy(), X=z.copy(),
                       Mi=np.zeros((2, 2)), Si=np.zeros((2, 2))))

    cur = old.copy()                            # current means (new for done nodes)
    for i in range(n):
        for t in range(T):
            s = st[t]
            B, Lp, Wp, Gp, Xp, Mip, Sip = s["B"], s["L"], s["W"], s["G"], s["X"], s["Mi"], s["Si"]
            has_prev, has_next = i > 0, i + 1 < n
            # g_i: observation terms of every j not in {i-1, i} + AR terms
            z = (Y[i, :, t, :].astype(np.float64)) @ Ri.T
            g = np.zeros(d)
            for j in range(n):
                if j == i or (has_prev and j == i - 1):
                    continue
                g += _J(cur[j, t], r).T @ z[j]
            if t > 0:
                g += QiPhi @ cur[i, t - 1]
            if t < T - 1:
                g += PhiTQi @ cur[i, t + 1]
            gA = np.zeros(d)
            gA[:2] = g[:2]
            J = _J(cur[i - 1, t], r) if has_prev else np.zeros((2, d))
            Jn = _J(old[i + 1, t], r) if has_next else np.zeros((2, d))
            zp = z[i - 1] if has_prev else np.zeros(2)
            yp = Y[i, i - 1, t, :].astype(np.float64) if has_prev else np.zeros(2)
            # base products (helper waves, one step ahead in the kernel)
            kj, v, vA, yv = B @ J.T, B @ g, B @ gA, B @ Jn.T
            ny = Jn @ yv
            # the one critical reduction round + the off-path dots
            a1, a2, c = Wp.T @ J.T, Xp.T @ J.T, J @ kj
            e, eA, jy = J @ v, J @ vA, J @ yv
            b1, b2, b1A, b2A = Wp.T @ g, Xp.T @ g, Wp.T @ gA, Xp.T @ gA
            f1, f2 = Wp.T @ Jn.T, Xp.T @ Jn.T
            # lane-local assembly
            W = kj - Lp @ a1 + Gp @ a2                       # = K_i J^T
            u = v - Lp @ b1 + Gp @ b2                        # = K_i g
            uA = vA - Lp @ b1A + Gp @ b2A                    # = K_i g^A
            kn = yv - Lp @ f1 + Gp @ f2                      # = K_i Jn^T
            if has_prev:
                JW = c - a1.T @ Mip @ a1 + a2.T @ Sip @ a2
                Mm = Rm + 0.5 * (JW + JW.T)
                Mi = _inv2(Mm)
                Ju = e - a1.T @ Mip @ b1 + a2.T @ Sip @ b2
                JuA = eA - a1.T @ Mip @ b1A + a2.T @ Sip @ b2A
                if variant != "bad":
                    mus = u + W @ (Mi @ (yp - Ju))
                else:
                    # rows 0,1 from P^-1 h^A, rows 2.. from P^-1 h^X (C off-blocks zeroed)
                    KE = np.zeros((d, 2))                   # K_i[:, 0:2]
                    KE[:] = B[:, :2] - Lp @ Wp[:2, :].T + Gp @ Xp[:2, :].T
                    WE = W[:2, :]                            # (J K_i E)^T = W_i rows 0,1
                    tA = uA + KE @ zp
                    jA = JuA + WE.T @ zp
                    uX = u - uA
                    tX = uX + W @ zp - KE @ zp
                    jX = (Ju - JuA) + JW @ zp - WE.T @ zp
                    mA = tA - W @ (Mi @ jA)
                    mX = tX - W @ (Mi @ jX)
                    mus = np.concatenate([mA[:2], mX[2:]])
                wn = jy - a1.T @ Mip @ f1 + a2.T @ Sip @ f2  # W_i^T Jn^T
                L = W @ Mi
            else:
                Mi = np.zeros((2, 2))
                W = np.zeros((d, 2))
                L = np.zeros((d, 2))
                wn = np.zeros((2, 2))
                if variant != "bad":
                    mus = u
                else:
                    mus = np.concatenate([uA[:2], (u - uA)[2:]])
            h = g + J.T @ zp
            if variant != "naive":
                mus = mus + 1e-6 * h
            if has_next:
                X = kn - L @ wn
                JnKJn = ny - f1.T @ Mip @ f1 + f2.T @ Sip @ f2
                JnX = JnKJn - wn.T @ Mi @ wn
                Sm = Rm - 0.5 * (JnX + JnX.T)
                Si = _inv2(Sm)
                G = X @ Si
            else:
                X = np.zeros((d, 2))
                Si = np.zeros((2, 2))
                G = np.zeros((d, 2))
            # outputs: damped mean (fp32 ops on the fp32-rounded solution)
            mu32 = mus.astype(f32)
            Xm[i, t] = lr32 * mu32 + om32 * Xm[i, t]
            cur[i, t] = Xm[i, t].astype(np.float64)
            K = B - Lp @ Wp.T + Gp @ Xp.T                   # K_i (helpers: base of step i+1)
            C = K - L @ W.T                                  # P_i^-1
            if variant == "naive":
                Pd = np.diag(np.linalg.inv(C))               # diag P_i
                c32 = np.diag(f32(1.0) / (Pd.astype(f32) + f32(1e-8)))
            else:
                Cl = np.tril(C)
                C = Cl + np.tril(C, -1).T                    # lower triangle mirrored
                if variant == "bad":
                    C[:2, 2:] = 0.0
                    C[2:, :2] = 0.0
                c32 = C.astype(f32) + np.eye(d, dtype=f32) * f32(1e-6)
            Xc[i, t] = lr32 * c32 + om32 * Xc[i, t]
            s.update(B=K, L=L, W=W, G=G, X=X, Mi=Mi, Si=Si)


CASES = [(12, 5, 2, "good", 0.5), (10, 4, 3, "bad", 1.0), (9, 3, 2, "naive", 0.3),
         (2, 3, 2, "good", 1.0), (7, 1, 1, "bad", 0.7), (1, 4, 2, "good", 1.0),
         (14, 6, 4, "good", 0.01), (11, 2, 3, "naive", 1.0)]


@pytest.mark.parametrize("n,T,r,variant,lr", CASES)
def test_lazy_rank4_sweep_matches_oracle(n, T, r, variant, lr):
    rng = np.random.default_rng(n * 100 + T * 10 + r)
    params = O.model_params(r, dtype=np.float64)
    d = 2 + 2 * r
    Y = rng.standard_normal((n, n, T, 2))
    for t in range(T):
        for i in range(n):
            Y[i, i, t] = 0.0
            for j in range(i):
                Y[i, j, t] = Y[j, i, t][::-1]
    Xm = (0.5 * rng.standard_normal((n, T, d))).astype(np.float32)
    A = 0.01 * rng.standard_normal((n, T, d, d))
    Xc = (0.5 * (A + A.transpose(0, 1, 3, 2)) + 0.6 * np.eye(d)).astype(np.float32)
    Xm_ref, Xc_ref = Xm.astype(np.float64), Xc.astype(np.float64)
    Xm2, Xc2 = Xm.copy(), Xc.copy()
    for _ in range(2):
        O.sweep(Y, Xm_ref, Xc_ref, params, variant, lr)
        sweep_lazy(Y.astype(np.float32), Xm2, Xc2, params, variant, lr)
    scale = max(1.0, np.abs(Xm_ref).max())
    assert np.abs(Xm2 - Xm_ref).max() <= 3e-6 * scale
    assert np.abs(Xc2 - Xc_ref).max() <= 1e-6 * max(1.0, np.abs(Xc_ref).max())


def test_wave_reduce_scatter_index_model():
    """CPU model of ame_wave.h's reduce-scatter bookkeeping: for every value
    count NV <= 64 each index is owned by exactly one of the 64 lanes (odd
    stages pad the upper half; pad slots must not alias real indices)."""
    for NV in range(1, 65):
        owners = {}
        for lane in range(64):
            idx, cnt, C = 0, NV, NV
            for S in range(6):
                H = (C + 1) // 2
                if (lane >> (5 - S)) & 1:
                    idx += H
                    cnt = max(cnt - H, 0)
                else:
                    cnt = min(cnt, H)
                C = H
            if cnt >= 1:
                assert idx not in owners, (NV, idx)
                owners[idx] = lane
        assert sorted(owners) == list(range(NV))
