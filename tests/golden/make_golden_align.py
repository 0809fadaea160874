"""Golden fixtures for the post-fit alignment from the reference.

TEST INFRASTRUCTURE ONLY.  Runs in the build container, where the reference
(Alfieriek/Python-Temporal-AME-SVI) is mounted read-only at /root/reference;
imports its own alignment utilities and writes plain-data ``.npz`` files
(inputs + expected outputs).  Nothing here ships; the GPU box never reads the
reference.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_align.py

Reference functions exercised (src/utils/alignment.py):
  * procrustes_alignment          :31-100
  * align_signs                   :103-164
  * align_latent_positions        :167-221
  * align_temporal_states         :224-321  (align_each_time True and False)
  * compute_alignment_error       :324-385
  * compute_correlation_after_alignment :388-436
"""
import os
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

sys.dont_write_bytecode = True
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from src.utils.alignment import (align_temporal_states, compute_alignment_error,  # noqa: E402
                                 compute_correlation_after_alignment)


def rotated_noisy(X, r, seed, noise=0.05):
    """A synthetic estimate: per-t random orthogonal mixing of U and V, row sign
    flips and noise -- what alignment is meant to undo."""
    rng = np.random.default_rng(seed)
    n, T, d = X.shape
    out = X.copy()
    for t in range(T):
        for blk in (slice(2, 2 + r), slice(2 + r, 2 + 2 * r)):
            q, _ = np.linalg.qr(rng.standard_normal((r, r)))
            out[:, t, blk] = X[:, t, blk] @ q
    flip = rng.random((n, T)) < 0.3
    out[:, :, :2][flip] *= -1
    out += noise * rng.standard_normal(out.shape)
    return out.astype(np.float32)


def run(tag, X_true, ests, r):
    res = {"X_true": X_true, "r": np.int64(r)}
    Xt = torch.from_numpy(X_true)
    for name, Xe in ests.items():
        Xe_t = torch.from_numpy(Xe)
        res[f"{name}_est"] = Xe
        res[f"{name}_each"] = align_temporal_states(Xe_t, Xt, r, align_each_time=True).numpy()
        res[f"{name}_global"] = align_temporal_states(Xe_t, Xt, r, align_each_time=False).numpy()
        err, _ = compute_alignment_error(Xe_t, Xt, latent_dim=r, align=True)
        err_na, _ = compute_alignment_error(Xe_t, Xt, latent_dim=r, align=False)
        res[f"{name}_err"] = np.float64(err)
        res[f"{name}_err_noalign"] = np.float64(err_na)
        res[f"{name}_corr"] = np.float64(compute_correlation_after_alignment(Xe_t, Xt, r))
    np.savez_compressed(os.path.join(OUT, f"{tag}_align.npz"), **res)
    print("wrote", tag, sorted(res))


def main():
    c1 = np.load(os.path.join(OUT, "c1_model.npz"))
    demo = np.load(os.path.join(OUT, "c1_demo100.npz"))
    run("c1", c1["X_true"], {m: demo[f"{m}_mean"] for m in ("good", "bad", "naive")}, 2)
    mid = np.load(os.path.join(OUT, "mid_model.npz"))
    run("mid", mid["X_true"], {"rot": rotated_noisy(mid["X_true"], 3, 1)}, 3)
    rng = np.random.default_rng(7)
    Xw = rng.standard_normal((64, 5, 34)).astype(np.float32)
    run("wide", Xw, {"rot": rotated_noisy(Xw, 16, 2, noise=0.2)}, 16)


if __name__ == "__main__":
    main()
