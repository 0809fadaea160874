"""Method comparison after fit: the reference's
``src/utils/diagnostics.py`` reporting used by demo.py (:176) and the
integration tests, with the same prints.  The state error is computed on the
device the estimates live on."""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch


def compute_state_prediction_error(X_true: torch.Tensor, X_pred: torch.Tensor) -> float:
    """diagnostics.py:254-273: mean squared state error."""
    X_pred = X_pred.to(X_true.device)
    return ((X_true - X_pred) ** 2).mean().item()


def compare_methods(results: Dict[str, Dict[str, Any]], metric: str = "reconstruction_error",
                    X_true: Optional[torch.Tensor] = None) -> None:
    """diagnostics.py:374-443: rank methods by the final `metric`, by state MSE,
    and print the improvement over the worst one."""
    print("\n" + "=" * 70)
    print("Method Comparison")
    print("=" * 70)
    scores = {name: res["history"][metric][-1] for name, res in results.items()
              if metric in res["history"] and len(res["history"][metric]) > 0}
    ranked = sorted(scores.items(), key=lambda x: x[1])
    print(f"\nFinal {metric}:")
    for rank, (name, score) in enumerate(ranked, 1):
        print(f"  {rank}. {name:20s}: {score:.6f}")
    if X_true is not None:
        print("\nState prediction MSE:")
        errs = {name: compute_state_prediction_error(X_true, res["X_est"])
                for name, res in results.items() if "X_est" in res}
        for rank, (name, err) in enumerate(sorted(errs.items(), key=lambda x: x[1]), 1):
            print(f"  {rank}. {name:20s}: {err:.6f}")
    if len(ranked) > 1:
        base_name, base = ranked[-1]
        print(f"\nImprovement over {base_name}:")
        for name, score in ranked[:-1]:
            print(f"  {name:20s}: {(1 - score / base) * 100:+.1f}%")
    print("=" * 70)
