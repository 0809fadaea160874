"""TEST INFRASTRUCTURE: the ELBO / MSE of a state at the large BASELINE shapes.

The same formulas as oracle/ame_oracle.py (expected_loglik, log_prior_initial,
log_prior_transitions, entropy, recon_error; structured_mf.py:115-209,
naive_mf.py:114-191, temporal_ame.py:255-291), evaluated with batched fp64
torch ops on the CPU (multithreaded), so n = 4096 runs in seconds instead of
minutes.  tests/test_elbo_check.py checks it against the oracle on the CPU.
Nothing here runs on the GPU.
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


def elbo_and_mse(Y, X_mean, X_cov, params, variant):
    """Y (n, n, T, 2), X_mean (n, T, d), X_cov (n, T, d, d) (numpy or torch,
    any float dtype) -> dict(loglik, prior0, trans, entropy, elbo, recon)."""
    Y = torch.as_tensor(Y)
    Xm = torch.as_tensor(X_mean).double()
    Xc = torch.as_tensor(X_cov)
    n, T, d = Xm.shape
    r = (d - 2) // 2
    P = {k: torch.as_tensor(v).double() for k, v in params.items()}
    Ri = P["R_inv"]
    logdetR = float(torch.logdet(P["R"]))
    trRi = float(torch.trace(Ri))
    upper = torch.triu(torch.ones(n, n, dtype=torch.bool), 1)
    off = ~torch.eye(n, dtype=torch.bool)
    quad = sq = trsum = 0.0
    for t in range(T):
        e = Y[:, :, t].double() - _mean_t(Xm[:, t], r)
        e0, e1 = e[..., 0], e[..., 1]
        qf = Ri[0, 0] * e0 * e0 + (Ri[0, 1] + Ri[1, 0]) * e0 * e1 + Ri[1, 1] * e1 * e1
        quad += float(qf[upper].sum())
        sq += float((e0 * e0 + e1 * e1)[off].sum())
        trsum += float(torch.diagonal(Xc[:, t].double(), dim1=-2, dim2=-1).sum())
    npairs = T * n * (n - 1) / 2.0
    corr = 0.0 if variant == "naive" else 0.1 * trRi / d * (n - 1) * trsum
    loglik = -0.5 * (npairs * (logdetR + 2 * LOG2PI) + quad + corr)
    S0 = torch.zeros(d, d, dtype=torch.float64)
    S0[:2, :2] = P["Sigma"]
    S0[2:, 2:] = P["Psi"]
    S0i = torch.linalg.inv(S0)
    mu0 = Xm[:, 0]
    prior0 = float((-0.5 * (torch.logdet(S0) + torch.einsum("na,ab,nb->n", mu0, S0i, mu0)
                            + torch.einsum("ab,nba->n", S0i, Xc[:, 0].double())
                            + d * LOG2PI)).sum())
    trans = 0.0
    if T > 1:
        Qi = torch.linalg.inv(P["Q"])
        res = Xm[:, 1:] - torch.einsum("ab,ntb->nta", P["Phi"], Xm[:, :-1])
        trq = torch.stack([torch.einsum("ab,nba->n", Qi, Xc[:, t].double()) for t in range(1, T)], 1)
        trans = float((-0.5 * (torch.logdet(P["Q"]) + torch.einsum("nta,ab,ntb->nt", res, Qi, res)
                               + trq + d * LOG2PI)).sum())
    ent = 0.0
    for t in range(T):
        sign, ld = torch.linalg.slogdet(Xc[:, t].double())
        ld = torch.where(sign > 0, ld, torch.where(sign == 0, torch.full_like(ld, -math.inf),
                                                    torch.full_like(ld, math.nan)))
        ent += float((0.5 * (d * (1 + LOG2PI) + ld)).sum())
    return {"loglik": loglik, "prior0": prior0, "trans": trans, "entropy": ent,
            "elbo": loglik + prior0 + trans + ent, "recon": sq / (n * (n - 1) * T)}
