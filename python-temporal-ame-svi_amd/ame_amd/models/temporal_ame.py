"""Temporal AME model: the inputs of the VI hot path.

Mirrors the reference's ``TemporalAMEModel`` (src/models/temporal_ame.py:25-362,
with the pieces it inherits from StaticAMEModel, static_ame.py:30-324, and
BaseAMEModel, models/base.py:24-196) so that either model object can be handed
to :class:`ame_amd.inference.TemporalAMEStructuredMFVI`.

Two generators:

* :meth:`generate_data` -- reference-identical stream.  Same seeding
  (models/base.py:73-74), same ``MultivariateNormal`` scale factors and the same
  order of ``normal_()`` draws as temporal_ame.py:172-216, so ``Y`` and ``X``
  are bit-identical to the reference for the same seed (pinned by
  tests/test_model.py against tests/golden).  O(n^2 T) Python; small configs.
* :meth:`generate_data_fast` -- vectorised, optionally on the GPU.  Same
  distribution, different random stream (documented in DESIGN.md); used for the
  benchmark configs where the reference generator would take ~40 min.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
from torch.distributions import MultivariateNormal


def _cov_matrix(dim: int, correlation: float, variance: float) -> torch.Tensor:
    """BaseAMEModel._generate_covariance_matrix (models/base.py:123-153)."""
    cov = torch.ones(dim, dim) * correlation * variance
    cov.diagonal().copy_(torch.ones(dim) * variance)
    return cov


def _block_diag_cov(sizes, corrs, variances) -> torch.Tensor:
    """BaseAMEModel._block_diagonal_covariance (models/base.py:155-196)."""
    total = sum(sizes)
    cov = torch.zeros(total, total)
    s = 0
    for size, c, v in zip(sizes, corrs, variances):
        cov[s:s + size, s:s + size] = _cov_matrix(size, c, v)
        s += size
    return cov



def fma_f32(p: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """fp32 fused multiply-add result p + s rounded ONCE to fp32, for p an
    exact fp64 product of two fp32 values and s fp32.  The fp64 sum is rounded
    first, so a plain ``.float()`` would round twice; the fp64 rounding error
    (TwoSum, exact) decides the halfway cases: when the fp64 sum lies exactly
    midway between two fp32 values and the error is non-zero, the true sum is
    on the error's side, and the sum is moved one fp64 ulp there before the
    fp32 rounding (no other fp32 rounding boundary lies within one fp64 ulp)."""
    s64 = s.double()
    t = p + s64
    bp = t - s64
    err = (p - bp) + (s64 - (t - bp))
    f = t.float()
    fd = f.double()
    toward = torch.where(t > fd, torch.full_like(f, float("inf")), torch.full_like(f, float("-inf")))
    mid = (fd + torch.nextafter(f, toward).double()) * 0.5
    tie = (t == mid) & (t != fd) & (err != 0)
    if bool(tie.any()):
        step = torch.where(err > 0, torch.full_like(t, float("inf")), torch.full_like(t, float("-inf")))
        t = torch.where(tie, torch.nextafter(t, step), t)
        f = t.float()
    return f

class TemporalAMEModel:
    """Temporal AME model with AR(1) latent dynamics.

    Constructor arguments and attributes follow temporal_ame.py:93-127:
    ``n, r, T, d = 2 + 2r, R, R_inv, Sigma, Psi, Phi, Q, X, Y``.
    """

    def __init__(self, n_nodes: int, n_time: int, latent_dim: int = 2,
                 ar_coefficient: float = 0.8, rho_additive: float = 0.5,
                 rho_multiplicative: float = 0.3, rho_dyadic: float = 0.5,
                 process_noise_scale: float = 0.1, seed: int = 42):
        # BaseAMEModel.__init__ (models/base.py:64-89): seed, then base R / swap Q
        torch.manual_seed(seed)
        np.random.seed(seed)
        self.seed = seed
        self.n = n_nodes
        self.r = latent_dim
        self.sigma, self.rho = 1.0, 0.0
        # StaticAMEModel.__init__ (static_ame.py:84-109): R overridden, var 0.1
        self.rho_additive = rho_additive
        self.rho_multiplicative = rho_multiplicative
        self.rho_dyadic = rho_dyadic
        self.R = _cov_matrix(2, rho_dyadic, 0.1)
        self.R_inv = torch.linalg.inv(self.R)
        self.Sigma = _cov_matrix(2, rho_additive, 1.0)
        self.Psi = _block_diag_cov([latent_dim, latent_dim],
                                   [rho_multiplicative, rho_multiplicative], [1.0, 1.0])
        # TemporalAMEModel.__init__ (temporal_ame.py:114-127)
        self.T = n_time
        self.ar_coefficient = ar_coefficient
        self.process_noise_scale = process_noise_scale
        self.d = 2 + 2 * self.r
        self._initialize_dynamics()
        self.A = None
        self.M = None
        self.X: Optional[torch.Tensor] = None
        self.Y: Optional[torch.Tensor] = None

    # temporal_ame.py:129-145
    def _initialize_dynamics(self) -> None:
        self.Phi = torch.eye(self.d) * self.ar_coefficient
        S = torch.zeros(self.d, self.d)
        S[:2, :2] = self.Sigma
        S[2:, 2:] = self.Psi
        self.Q = (1 - self.ar_coefficient ** 2) * S
        self.Q = self.Q * self.process_noise_scale

    def sigma0(self) -> torch.Tensor:
        S = torch.zeros(self.d, self.d)
        S[:2, :2] = self.Sigma
        S[2:, 2:] = self.Psi
        return S

    # ------------------------------------------------------------------
    # generators
    # ------------------------------------------------------------------
    def generate_data(self, return_latents: bool = False, X: Optional[torch.Tensor] = None):
        """Reference-identical generator (temporal_ame.py:147-220).

        ``X`` (optional, (n, T, d)): take these latent trajectories instead of
        forming them, while consuming exactly the random draws the reference
        spends on them.  The reference forms X with small MKL matvecs whose
        rounding depends on the host CPU's code path; given X, the observations
        below are bit-identical on any host (tests/test_reference_c2.py checks
        both against the reference's own run)."""
        n, T, d = self.n, self.T, self.d
        self.Y = torch.zeros(n, n, T, 2)
        L0 = MultivariateNormal(torch.zeros(d), self.sigma0())._unbroadcasted_scale_tril
        LQ = MultivariateNormal(torch.zeros(d), self.Q)._unbroadcasted_scale_tril
        LR = MultivariateNormal(torch.zeros(2), self.R)._unbroadcasted_scale_tril
        z_d = torch.zeros(d)

        def sample(L, loc, k):   # MultivariateNormal.rsample with one normal_() draw
            eps = torch.empty(k).normal_()
            return loc + torch.matmul(L, eps.unsqueeze(-1)).squeeze(-1)

        if X is None:
            self.X = torch.zeros(n, T, d)
            for i in range(n):
                self.X[i, 0] = sample(L0, z_d, d)
                for t in range(1, T):
                    self.X[i, t] = torch.matmul(self.Phi, self.X[i, t - 1]) + sample(LQ, z_d, d)
        else:
            self.X = torch.as_tensor(X, dtype=torch.float32).clone()
            if tuple(self.X.shape) != (n, T, d):
                raise ValueError(f"X has shape {tuple(self.X.shape)}, expected {(n, T, d)}")
            scratch = torch.empty(d)
            for _ in range(n * T):   # the same draws, in the same order
                scratch.normal_()
        # Observation noise (temporal_ame.py:203-214): one 2-vector draw per
        # upper-triangle dyad, t-major then i then j.  A CPU normal_() call on
        # fewer than 16 floats takes the scalar Box-Muller path, which caches the
        # pair's second value, so calls of 14 floats (7 dyads) consume the stream
        # exactly like 7 calls of 2.  L R^{1/2} eps with the lower-triangular
        # factor is [L00 e0, L11 e1 + L10 e0] rounded as the reference's 2x2 matvec
        # rounds it (the second entry as one fused multiply-add onto the rounded
        # L10 e0 product), checked bit for bit against the reference's Y.
        iu = torch.triu_indices(n, n, 1)
        npairs = iu.shape[1]
        eps = torch.empty(npairs * 2)
        l00, l10, l11 = (float(LR[0, 0]), float(LR[1, 0]), float(LR[1, 1]))
        for t in range(T):
            for k in range(0, npairs * 2, 14):
                eps[k:k + 14].normal_()
            e = eps.view(npairs, 2).double()
            p0 = (l00 * e[:, 0]).float()
            p10 = (l10 * e[:, 0]).float()
            p1 = fma_f32(l11 * e[:, 1], p10)
            mu_t = self._mean_seqfma(self.X[:, t, :2], self.X[:, t, 2:])
            dy = mu_t[iu[0], iu[1]] + torch.stack([p0, p1], dim=1)
            self.Y[iu[0], iu[1], t] = dy
            self.Y[iu[1], iu[0], t, 0] = dy[:, 1]
            self.Y[iu[1], iu[0], t, 1] = dy[:, 0]
        if return_latents:
            return self.Y, self.X
        return self.Y

    def _mean_seqfma(self, A: torch.Tensor, M: torch.Tensor) -> torch.Tensor:
        """compute_mean (static_ame.py:189-238) of one slice with U V^T summed as
        the reference's fp32 sgemm sums it on the fixture host (MKL: one fused
        multiply-add per k, k ascending; measured bit-exact), but independent of
        the host's BLAS: each step is an exact fp64 product plus the running fp32
        sum, rounded once to fp32 (:func:`fma_f32`)."""
        a, b = A[:, 0], A[:, 1]
        U, V = M[:, :self.r].double(), M[:, self.r:].double()
        mult = torch.zeros(A.shape[0], A.shape[0], dtype=torch.float32)
        for k in range(self.r):
            mult = fma_f32(torch.outer(U[:, k], V[:, k]), mult)
        additive = a.unsqueeze(1) + b.unsqueeze(0)
        mu = torch.zeros(A.shape[0], A.shape[0], 2)
        mu[:, :, 0] = additive + mult
        mu[:, :, 1] = additive.t() + mult.t()
        return mu

    def generate_data_fast(self, return_latents: bool = False, device=None,
                           seed: Optional[int] = None):
        """Vectorised generator: same distribution as :meth:`generate_data`,
        different random stream.  ``device='cuda'`` builds Y in HBM."""
        n, T, d = self.n, self.T, self.d
        dev = torch.device(device) if device is not None else torch.device("cpu")
        g = torch.Generator(device=dev)
        g.manual_seed(self.seed if seed is None else seed)
        L0 = torch.linalg.cholesky(self.sigma0()).to(dev)
        LQ = torch.linalg.cholesky(self.Q).to(dev)
        LR = torch.linalg.cholesky(self.R).to(dev)
        Phi = self.Phi.to(dev)
        X = torch.empty(n, T, d, device=dev)
        X[:, 0] = torch.randn(n, d, generator=g, device=dev) @ L0.T
        for t in range(1, T):
            X[:, t] = X[:, t - 1] @ Phi.T + torch.randn(n, d, generator=g, device=dev) @ LQ.T
        Y = torch.empty(n, n, T, 2, device=dev)
        iu = torch.triu_indices(n, n, 1, device=dev)
        for t in range(T):
            mu = self.compute_mean(X[:, t, :2], X[:, t, 2:])
            noise = torch.randn(n, n, 2, generator=g, device=dev) @ LR.T
            dy = mu + noise
            Yt = torch.zeros(n, n, 2, device=dev)
            Yt[iu[0], iu[1]] = dy[iu[0], iu[1]]
            Yt[iu[1], iu[0], 0] = dy[iu[0], iu[1], 1]
            Yt[iu[1], iu[0], 1] = dy[iu[0], iu[1], 0]
            Y[:, :, t] = Yt
        self.X, self.Y = X, Y
        if return_latents:
            return Y, X
        return Y

    # ------------------------------------------------------------------
    # model functions (static_ame.py:189-238, temporal_ame.py:222-313)
    # ------------------------------------------------------------------
    def compute_mean(self, A: torch.Tensor, M: torch.Tensor) -> torch.Tensor:
        n = A.shape[0]
        mu = torch.zeros(n, n, 2, dtype=A.dtype, device=A.device)
        a, b = A[:, 0], A[:, 1]
        U, V = M[:, :self.r], M[:, self.r:]
        additive = a.unsqueeze(1) + b.unsqueeze(0)
        multiplicative = torch.matmul(U, V.t())
        mu[:, :, 0] = additive + multiplicative
        mu[:, :, 1] = additive.t() + multiplicative.t()
        return mu

    def get_states_at_time(self, t: int) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.X is None:
            raise ValueError("No data generated yet. Call generate_data() first.")
        if t < 0 or t >= self.T:
            raise ValueError(f"Time index {t} out of bounds [0, {self.T}).")
        return self.X[:, t, :2], self.X[:, t, 2:]

    def compute_temporal_reconstruction_error(self, X_est: torch.Tensor) -> float:
        """Mean squared error over t and i != j (temporal_ame.py:255-291)."""
        if self.Y is None:
            raise ValueError("No data generated yet. Call generate_data() first.")
        X_est = X_est.to(self.Y.device)
        total = 0.0
        mask = 1 - torch.eye(self.n, device=self.Y.device).unsqueeze(-1)
        for t in range(self.T):
            mu = self.compute_mean(X_est[:, t, :2], X_est[:, t, 2:])
            total += (((self.Y[:, :, t] - mu) ** 2) * mask).sum().item()
        return total / (self.n * (self.n - 1) * self.T)

    def compute_state_prediction_error(self, X_est: torch.Tensor) -> float:
        if self.X is None:
            raise ValueError("No data generated yet. Call generate_data() first.")
        return ((self.X - X_est.to(self.X.device)) ** 2).mean().item()
