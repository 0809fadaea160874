"""Template-method VI base classes (reference: src/inference/base.py:23-343).

Same constructor, ``fit`` loop, convergence rule (relative ELBO change below
``tolerance`` for 3 consecutive iterations, base.py:183-191), history dict and
progress printing (base.py:162-164, 196-206, 335) as the reference, so a caller
of the reference finds the same behaviour.  Subclasses run the hooks on the GPU
through :class:`ame_amd.engine.DeviceEngine`.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Dict, List

import numpy as np
import torch


class BaseVariationalInference(ABC):
    """Abstract VI base (base.py:23-272)."""

    def __init__(self, model, learning_rate: float = 0.01, seed: int = 42):
        torch.manual_seed(seed)
        np.random.seed(seed)
        self.model = model
        self.Y = model.Y
        self.n = model.n
        self.lr = learning_rate
        self.history: Dict[str, List[float]] = {"elbo": [], "reconstruction_error": []}
        self._initialize_variational_params()

    @abstractmethod
    def _initialize_variational_params(self) -> None: ...

    @abstractmethod
    def _compute_elbo(self) -> float: ...

    @abstractmethod
    def _update_step(self) -> None: ...

    def fit(self, max_iter: int = 100, tolerance: float = 1e-4, verbose: bool = True,
            check_every: int = 10) -> Dict[str, List[float]]:
        """base.py:127-208, unchanged semantics."""
        if verbose:
            print(f"Starting {self.__class__.__name__} optimization...")
            print("=" * 60)
        converged = False
        patience_counter = 0
        prev_elbo = -np.inf
        ok = False
        try:
            for iteration in range(max_iter):
                self._fit_iteration(iteration, max_iter)
                self._update_step()
                elbo = self._compute_elbo()
                self.history["elbo"].append(elbo)
                recon_error = self._compute_reconstruction_error()
                self.history["reconstruction_error"].append(recon_error)
                if iteration > 0:
                    rel_change = abs(elbo - prev_elbo) / (abs(prev_elbo) + 1e-8)
                    if rel_change < tolerance:
                        patience_counter += 1
                    else:
                        patience_counter = 0
                    if patience_counter >= 3:
                        converged = True
                prev_elbo = elbo
                if verbose and (iteration % check_every == 0 or iteration == max_iter - 1):
                    self._print_progress(iteration, elbo, recon_error)
                if converged:
                    if verbose:
                        print(f"\nConverged at iteration {iteration}")
                    break
            ok = True
        finally:
            self._fit_end(ok)
        if verbose and not converged:
            print("\nReached maximum iterations without convergence")
        return self.history

    def _fit_iteration(self, iteration: int, max_iter: int) -> None:
        """Hook: fit() is about to run `iteration` of `max_iter` (no-op here)."""

    def _fit_end(self, ok: bool = True) -> None:
        """Hook: fit() is returning (ok) or raising (not ok); no-op here."""

    def _compute_reconstruction_error(self) -> float:
        if hasattr(self, "get_variational_means"):
            params = self.get_variational_means()
            return self.model.compute_reconstruction_error(*params)
        return 0.0

    def _print_progress(self, iteration: int, elbo: float, recon_error: float) -> None:
        print(f"Iter {iteration:4d} | ELBO: {elbo:10.2f} | MSE: {recon_error:.6f}")

    def get_elbo_history(self) -> List[float]:
        return self.history["elbo"]

    def get_reconstruction_history(self) -> List[float]:
        return self.history["reconstruction_error"]


class BaseTemporalVariationalInference(BaseVariationalInference):
    """base.py:275-343: sets T, d, r before the base init (init uses them)."""

    def __init__(self, model, learning_rate: float = 0.01, seed: int = 42):
        self.T = model.T
        self.d = model.d
        self.r = model.r
        super().__init__(model, learning_rate, seed)

    def _compute_reconstruction_error(self) -> float:
        if hasattr(self, "X_mean"):
            return self.model.compute_temporal_reconstruction_error(self.X_mean)
        return 0.0

    def _print_progress(self, iteration: int, elbo: float, recon_error: float) -> None:
        output = f"Iter {iteration:4d} | ELBO: {elbo:10.2f} | MSE: {recon_error:.6f}"
        if hasattr(self, "history") and "state_error" in self.history:
            if len(self.history["state_error"]) > 0:
                output += f" | State MSE: {self.history['state_error'][-1]:.6f}"
        print(output)
