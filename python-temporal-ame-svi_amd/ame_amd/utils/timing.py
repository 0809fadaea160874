"""Timing harness for one VI run.

``run_method_with_timing`` mirrors the reference's
``experiments/utils.py:146-229`` (same arguments, same result keys, same
prints) and adds what the device path can report on top: ``kernels_ms``, the
average duration per launch of each HIP kernel of the fit (HIP events recorded
on the streams the kernels run on), and ``iterations_per_s``.
"""
from __future__ import annotations

import time
from typing import Any, Dict

import torch


def run_method_with_timing(vi_class, model, method_name: str, max_iter: int = 100,
                           verbose: bool = True, **vi_kwargs) -> Dict[str, Any]:
    """experiments/utils.py:146-229 plus per-kernel device times."""
    if verbose:
        print(f"\n{'=' * 70}")
        print(f"Running: {method_name}")
        print(f"{'=' * 70}")
    vi = vi_class(model, **vi_kwargs)
    eng = getattr(vi, "engine", None)
    if eng is not None:
        eng.timing = True
        eng.events.clear()
    start_time = time.time()
    history = vi.fit(max_iter=max_iter, verbose=verbose)
    if eng is not None:
        torch.cuda.synchronize(eng.dev)
    runtime = time.time() - start_time
    if hasattr(vi, "X_mean"):
        X_est = vi.X_mean
    elif hasattr(vi, "get_variational_means"):
        X_est = vi.get_variational_means()
    else:
        X_est = None
    iters = len(history["elbo"]) if "elbo" in history else max_iter
    result = {
        "vi": vi,
        "history": history,
        "X_est": X_est,
        "runtime": runtime,
        "iterations": iters,
        "method_name": method_name,
        "iterations_per_s": iters / runtime if runtime > 0 else float("inf"),
    }
    if eng is not None:
        kms, _ = eng.kernel_ms()
        result["kernels_ms"] = kms
        eng.timing = False
    if verbose:
        print(f"\nCompleted in {runtime:.2f} seconds")
        if "reconstruction_error" in history:
            print(f"Final MSE: {history['reconstruction_error'][-1]:.6f}")
    return result
