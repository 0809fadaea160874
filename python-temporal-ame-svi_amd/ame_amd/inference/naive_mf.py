"""Naive mean-field VI for temporal AME on MI355X.

Drop-in for the reference ``TemporalAMENaiveMFVI`` (src/inference/naive_mf.py:29-396):
same sweep order as the structured variant, mean = solve(P, h) (naive_mf.py:268),
covariance = diag(1 / (diag P + 1e-8)) (:271-274), ELBO without the trace
correction (:130).  Runs on the same kernels with variant AME_NAIVE.
"""
from __future__ import annotations

import torch

from ._device_vi import DeviceTemporalVI


class TemporalAMENaiveMFVI(DeviceTemporalVI):
    _variant = "naive"

    def __init__(self, model, learning_rate: float = 1.0, init_scale: float = 0.1,
                 seed: int = 42, device=None, distributed=None, engine_options=None):
        self.init_scale = init_scale
        super().__init__(model, learning_rate, seed, device=device, distributed=distributed,
                         engine_options=engine_options)

    def _initialize_variational_params(self) -> None:
        """naive_mf.py:71-87 (no RNG draw for the covariances)."""
        n, T, d = self.n, self.T, self.d
        self.X_mean = torch.randn(n, T, d) * self.init_scale
        self.X_cov = (torch.eye(d) * 0.5).expand(n, T, d, d).contiguous()

    def predict_forward(self, n_steps: int = 1) -> torch.Tensor:
        """naive_mf.py:386-396: X_pred[i, s] = Phi^(s+1) X_mean[i, -1]."""
        Phi = self.model.Phi
        X_pred = torch.zeros(self.n, n_steps, self.d)
        last = self.X_mean[:, -1].clone()
        for i in range(self.n):
            x = last[i].clone()
            for s in range(n_steps):
                x = torch.matmul(Phi, x)
                X_pred[i, s] = x
        return X_pred
