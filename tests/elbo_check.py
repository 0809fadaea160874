"""TEST INFRASTRUCTURE: the ELBO / MSE of a state at the large BASELINE shapes.

The same formulas as oracle/ame_oracle.py (expected_loglik, log_prior_initial,
log_prior_transitions, entropy, recon_error; structured_mf.py:115-209,
naive_mf.py:114-191, temporal_ame.py:255-291), evaluated with batched fp64
torch ops on the CPU (multithreaded), so n = 4096 runs in seconds instead of
minutes.  The work is split by what it reads, one time slice at a time, so
that config 5 at full size (Y 34 GB, X_cov 18 GB) never needs a full host or
fp64 copy:

* :func:`cov_sums` -- everything that reads the covariances (trace sums, the
  prior traces, log-determinants), from a per-slice provider;
* :func:`pair_sums` -- everything that reads Y (the quadratic forms of the
  expected log-likelihood and the squared residuals of the MSE), from a
  per-slice provider, for several mean states in one pass over Y;
* :func:`assemble` -- the ELBO pieces from those sums and the means.

tests/test_elbo_check.py checks :func:`elbo_and_mse` (built from the three)
against the oracle on the CPU.  ``device=`` evaluates the same fp64 torch ops
elsewhere (config 5's full state: on the GPU, with torch's own kernels, pinned
to the CPU evaluation on sample slices in the same test).
"""
import math

import torch

LOG2PI = math.log(2.0 * math.pi)


def _mean_t(x, r):
    """compute_mean (static_ame.py:189-238) of one slice, fp64."""
    a, b = x[:, 0], x[:, 1]
    U, V = x[:, 2:2 + r], x[:, 2 + r:]
    add = a[:, None] + b[None, :]
    mult = U @ V.T
    return torch.stack([add + mult, add.T + mult.T], dim=-1)


def _params(params):
    return {k: torch.as_tensor(v).double() for k, v in params.items()}


def _S0(P, d):
    S0 = torch.zeros(d, d, dtype=torch.float64)
    S0[:2, :2] = P["Sigma"]
    S0[2:, 2:] = P["Psi"]
    return S0


def cov_sums(get_cov, T, params, device="cpu", ts=None):
    """get_cov(t) -> (n, d, d) covariances of slice t (any float dtype and
    device; evaluated on `device`).  Returns the fp64 sums the ELBO needs from
    the covariances, over all T slices or the slices `ts`."""
    P = _params(params)
    out = {"trsum": 0.0, "tr0": 0.0, "trq": 0.0, "ld": 0.0}
    S0i = Qi = None
    for t in (range(T) if ts is None else ts):
        C = torch.as_tensor(get_cov(t)).to(device).double()
        d = C.shape[-1]
        if S0i is None:
            S0i = torch.linalg.inv(_S0(P, d)).to(device)
            Qi = torch.linalg.inv(P["Q"]).to(device)
        out["trsum"] += float(torch.diagonal(C, dim1=-2, dim2=-1).sum())
        if t == 0:
            out["tr0"] += float(torch.einsum("ab,nba->", S0i, C))
        else:
            out["trq"] += float(torch.einsum("ab,nba->", Qi, C))
        sign, ld = torch.linalg.slogdet(C)
        ld = torch.where(sign > 0, ld, torch.where(sign == 0, torch.full_like(ld, -math.inf),
                                                    torch.full_like(ld, math.nan)))
        out["ld"] += float(ld.sum())
    return out


def pair_sums(get_y, means, params, device="cpu", ts=None):
    """get_y(t) -> (n, n, 2) observed slice t; means: list of (n, T, d) states.
    Returns [(quad, sq)] per state: the upper-triangle quadratic forms with R^-1
    and the off-diagonal squared residuals, summed over all slices (or `ts`),
    evaluated in fp64 on `device`."""
    P = _params(params)
    Ri = P["R_inv"]
    Xs = [torch.as_tensor(x).double() for x in means]
    n, T, d = Xs[0].shape
    r = (d - 2) // 2
    upper = torch.triu(torch.ones(n, n, dtype=torch.bool, device=device), 1)
    off = ~torch.eye(n, dtype=torch.bool, device=device)
    acc = [[0.0, 0.0] for _ in Xs]
    for t in (range(T) if ts is None else ts):
        Y = torch.as_tensor(get_y(t)).to(device).double()
        for k, Xm in enumerate(Xs):
            e = Y - _mean_t(Xm[:, t].to(device), r)
            e0, e1 = e[..., 0], e[..., 1]
            qf = Ri[0, 0] * e0 * e0 + (Ri[0, 1] + Ri[1, 0]) * e0 * e1 + Ri[1, 1] * e1 * e1
            acc[k][0] += float(qf[upper].sum())
            acc[k][1] += float((e0 * e0 + e1 * e1)[off].sum())
    return [tuple(a) for a in acc]


def assemble(X_mean, cs, quad, sq, params, variant):
    """ELBO pieces + MSE from the sums above and the means (n, T, d)."""
    Xm = torch.as_tensor(X_mean).double()
    n, T, d = Xm.shape
    P = _params(params)
    logdetR = float(torch.logdet(P["R"]))
    trRi = float(torch.trace(P["R_inv"]))
    npairs = T * n * (n - 1) / 2.0
    corr = 0.0 if variant == "naive" else 0.1 * trRi / d * (n - 1) * cs["trsum"]
    loglik = -0.5 * (npairs * (logdetR + 2 * LOG2PI) + quad + corr)
    S0 = _S0(P, d)
    S0i = torch.linalg.inv(S0)
    mu0 = Xm[:, 0]
    prior0 = -0.5 * (n * (float(torch.logdet(S0)) + d * LOG2PI)
                     + float(torch.einsum("na,ab,nb->", mu0, S0i, mu0)) + cs["tr0"])
    trans = 0.0
    if T > 1:
        Qi = torch.linalg.inv(P["Q"])
        res = Xm[:, 1:] - torch.einsum("ab,ntb->nta", P["Phi"], Xm[:, :-1])
        trans = -0.5 * (n * (T - 1) * (float(torch.logdet(P["Q"])) + d * LOG2PI)
                        + float(torch.einsum("nta,ab,ntb->", res, Qi, res)) + cs["trq"])
    ent = 0.5 * (n * T * d * (1 + LOG2PI) + cs["ld"])
    return {"loglik": loglik, "prior0": prior0, "trans": trans, "entropy": ent,
            "elbo": loglik + prior0 + trans + ent, "recon": sq / (n * (n - 1) * T)}


def elbo_and_mse(Y, X_mean, X_cov, params, variant):
    """Y (n, n, T, 2), X_mean (n, T, d), X_cov (n, T, d, d) (numpy or torch,
    any float dtype) -> dict(loglik, prior0, trans, entropy, elbo, recon)."""
    Y = torch.as_tensor(Y)
    Xc = torch.as_tensor(X_cov)
    T = Xc.shape[1]
    cs = cov_sums(lambda t: Xc[:, t], T, params)
    (quad, sq), = pair_sums(lambda t: Y[:, :, t], [X_mean], params)
    return assemble(X_mean, cs, quad, sq, params, variant)
