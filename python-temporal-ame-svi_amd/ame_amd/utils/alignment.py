"""Post-fit alignment of estimated and true state trajectories.

Same names, arguments and results as the reference's ``src/utils/alignment.py``
(Alfieriek/Python-Temporal-AME-SVI):

* ``align_temporal_states`` (:224-321) and ``compute_alignment_error``
  (:324-385) -- the per-time-step loops -- run on the GPU through
  ``libame_amd.so``: ``ame_align_cross`` forms every cross-product block
  ``A_true^T A_est`` in one pass over both trajectories, the host turns the
  small blocks into rotations (``R = U Vt`` of their SVD with the reference's
  reflection fix, :79-87), and ``ame_align_apply`` rotates, sign-aligns and
  writes every row and sums the squared error in the same pass;
* ``align_latent_positions`` (:167-221) and the static (n, d) case of
  ``compute_alignment_error`` reuse the same kernels with T = 1;
* ``procrustes_alignment`` (:31-100) and ``align_signs`` (:103-164) on single
  small matrices are plain tensor algebra on the input's device.

Inputs may live on the CPU (the reference's convention: ``vi.X_mean`` is a CPU
tensor) or on a GPU; the result is returned on the device ``X_est`` came from.
There is no CPU fallback for the kernel path: without a GPU it raises.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np
import torch

from .. import _lib

__all__ = ["procrustes_alignment", "align_signs", "align_latent_positions",
           "align_temporal_states", "compute_alignment_error",
           "compute_correlation_after_alignment"]


def _rotations(cross: np.ndarray) -> np.ndarray:
    """R = U Vt per block (batched), last row of Vt negated where det(R) < 0
    (alignment.py:79-87)."""
    U, _, Vt = np.linalg.svd(cross)
    R = U @ Vt
    neg = np.linalg.det(R) < 0
    if neg.any():
        Vt = Vt.copy()
        Vt[neg, -1, :] *= -1
        R = U @ Vt
    return R


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("ame_amd.utils.alignment: no GPU visible; the HIP path has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def _align_device(X_est: torch.Tensor, X_true: torch.Tensor, r: int,
                  align_each_time: bool) -> Tuple[torch.Tensor, float]:
    """(n, T, d) -> (aligned (n, T, d) on X_est's device, sum of squared errors)."""
    if X_est.shape != X_true.shape or X_est.ndim != 3:
        raise ValueError(f"shape mismatch: {tuple(X_est.shape)} vs {tuple(X_true.shape)}")
    n, T, d = (int(s) for s in X_est.shape)
    if d != 2 + 2 * r:
        raise ValueError(f"state dim {d} != 2 + 2 * latent_dim ({2 + 2 * r})")
    L = _lib.lib()
    if r not in _lib.supported_r():
        raise RuntimeError(f"ame_amd: latent_dim={r} not compiled (supported {_lib.supported_r()})")
    dev = X_est.device if X_est.is_cuda else _device()
    gm = 0 if align_each_time else 1
    with torch.cuda.device(dev):
        st = torch.cuda.current_stream(dev)
        xe = X_est.detach().to(dev, torch.float32).contiguous()
        xt = X_true.detach().to(dev, torch.float32).contiguous()
        ncross = int(L.ame_align_cross_size(n, T, r, gm))
        nwork = int(L.ame_align_work_size(n, T, r))
        npart = int(L.ame_align_partials_size(n, T))
        if min(ncross, nwork, npart) < 0:
            _lib.check(-1, "ame_align sizes")
        cross = torch.empty(ncross, dtype=torch.float64, device=dev)
        work = torch.empty(max(nwork, 1), dtype=torch.float64, device=dev)
        part = torch.empty(npart, dtype=torch.float64, device=dev)
        out = torch.empty_like(xe)
        sp = ctypes.c_void_p(st.cuda_stream)
        _lib.check(L.ame_align_cross(ctypes.c_void_p(xe.data_ptr()), ctypes.c_void_p(xt.data_ptr()),
                                     n, T, r, gm, ctypes.c_void_p(cross.data_ptr()),
                                     ctypes.c_void_p(work.data_ptr()), sp), "ame_align_cross")
        w = 2 * r if gm else r
        blocks = cross.cpu().numpy().reshape(-1, w, w)
        rot = torch.from_numpy(np.ascontiguousarray(_rotations(blocks))).to(dev)
        _lib.check(L.ame_align_apply(ctypes.c_void_p(xe.data_ptr()), ctypes.c_void_p(xt.data_ptr()),
                                     n, T, r, gm, ctypes.c_void_p(rot.data_ptr()),
                                     ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(part.data_ptr()), sp), "ame_align_apply")
        sq = float(part.sum().item())
    # the kernels compute in fp32; hand back the caller's dtype and device
    # (the reference returns X_est-typed results, alignment.py:275-321)
    return out.to(X_est.device, X_est.dtype), sq


def procrustes_alignment(X_est: torch.Tensor, X_true: torch.Tensor,
                         scaling: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """alignment.py:31-100 (R = U Vt of svd(X_true^T X_est), det fix, optional scale)."""
    M = X_true.t() @ X_est
    U, _, Vt = torch.linalg.svd(M)
    R = U @ Vt
    if torch.det(R) < 0:
        Vt = Vt.clone()
        Vt[-1, :] *= -1
        R = U @ Vt
    X_aligned = X_est @ R
    if scaling:
        num = torch.trace(X_true.t() @ X_aligned)
        den = torch.trace(X_aligned.t() @ X_aligned)
        if den > 1e-10:
            X_aligned = X_aligned * (num / den)
    return X_aligned, R


def align_signs(X_est: torch.Tensor, X_true: torch.Tensor, dim: int = -1) -> torch.Tensor:
    """alignment.py:103-164: flip each slice along `dim` (rows for the last
    dim) whose negation is closer to the target."""
    if dim == -1 or dim == X_est.ndim - 1:
        flat_e = X_est.reshape(X_est.shape[0], -1)
        flat_t = X_true.reshape(X_true.shape[0], -1)
        neg = torch.linalg.norm(-flat_e - flat_t, dim=1) < torch.linalg.norm(flat_e - flat_t, dim=1)
        shape = (-1,) + (1,) * (X_est.ndim - 1)
        return torch.where(neg.reshape(shape), -X_est, X_est)
    out = X_est.clone()
    for i in range(X_est.shape[dim]):
        e = X_est.select(dim, i)
        t = X_true.select(dim, i)
        if torch.linalg.norm(-e - t) < torch.linalg.norm(e - t):
            out.select(dim, i).neg_()
    return out


def align_latent_positions(M_est: torch.Tensor, M_true: torch.Tensor,
                           latent_dim: int) -> torch.Tensor:
    """alignment.py:167-221 on the GPU (one time step of the temporal kernels)."""
    n = M_est.shape[0]
    pad = M_est.new_zeros((n, 1, 2))
    Xe = torch.cat([pad, M_est.reshape(n, 1, -1)], dim=2)
    Xt = torch.cat([pad, M_true.reshape(n, 1, -1).to(M_est.dtype)], dim=2)
    out, _ = _align_device(Xe, Xt, latent_dim, True)
    return out[:, 0, 2:].to(M_est.dtype)


def align_temporal_states(X_est: torch.Tensor, X_true: torch.Tensor, latent_dim: int,
                          align_each_time: bool = True) -> torch.Tensor:
    """alignment.py:224-321 on the GPU."""
    out, _ = _align_device(X_est, X_true, latent_dim, align_each_time)
    return out


def compute_alignment_error(X_est: torch.Tensor, X_true: torch.Tensor,
                            latent_dim: Optional[int] = None,
                            align: bool = True) -> Tuple[float, torch.Tensor]:
    """alignment.py:324-385: mean squared error after (optional) alignment."""
    if align:
        if X_est.ndim == 3:
            if latent_dim is None:
                raise ValueError("latent_dim must be provided for temporal alignment")
            X_aligned, sq = _align_device(X_est, X_true, latent_dim, True)
            return sq / X_est.numel(), X_aligned
        if X_est.ndim == 2:
            if latent_dim is not None:
                n = X_est.shape[0]
                X_aligned, sq = _align_device(X_est.reshape(n, 1, -1), X_true.reshape(n, 1, -1),
                                              latent_dim, True)
                return sq / X_est.numel(), X_aligned.reshape(X_est.shape)
            X_aligned = align_signs(X_est, X_true, dim=1)
        else:
            X_aligned = X_est
    else:
        X_aligned = X_est
    error = ((X_aligned - X_true) ** 2).mean().item()
    return error, X_aligned


def compute_correlation_after_alignment(X_est: torch.Tensor, X_true: torch.Tensor,
                                        latent_dim: Optional[int] = None) -> float:
    """alignment.py:388-436: Pearson correlation of the aligned estimate."""
    _, X_aligned = compute_alignment_error(X_est, X_true, latent_dim, align=True)
    a = X_aligned.flatten().double()
    b = X_true.flatten().double().to(a.device)
    a = a - a.mean()
    b = b - b.mean()
    den = torch.sqrt((a ** 2).sum() * (b ** 2).sum())
    if den < 1e-10:
        return 0.0
    return float(((a * b).sum() / den).item())
