"""Bit-for-bit comparison of two library builds on one fit (GPU box).

    AME_LIB_PATH=libA.so python tools/bitcmp.py save A.npz [n,T,r] [variant] [iters] [kind]
    AME_LIB_PATH=libB.so python tools/bitcmp.py save B.npz ...
    python tools/bitcmp.py cmp A.npz B.npz

A kernel change meant to keep every sum (same products, same order) must give
equal means and covariances; `cmp` prints the first differing entries otherwise.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))


def save(path, shape="4096,4,32", variant="good", iters="2", kind=None):
    import torch
    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    n, T, r = (int(x) for x in shape.split(","))
    dev = torch.device("cuda", 0)
    m = TemporalAMEModel(n, T, r, seed=5)
    m.generate_data_fast(seed=6)
    opts = {} if kind is None else {"sweep_kernel": int(kind)}
    if variant == "naive":
        vi = TemporalAMENaiveMFVI(m, learning_rate=0.5, device=dev, engine_options=opts)
    else:
        vi = TemporalAMEStructuredMFVI(m, factorization=variant, learning_rate=0.5, device=dev,
                                       engine_options=opts)
    vi.fit(max_iter=int(iters), tolerance=0.0, verbose=False)
    import hashlib
    cov = vi.X_cov.numpy()
    # covariances as a digest plus their diagonal (the full array is GBs at scale)
    np.savez(path, mean=vi.X_mean.numpy(), covdiag=np.diagonal(cov, axis1=-2, axis2=-1).copy(),
             covsha=np.frombuffer(hashlib.sha256(cov.tobytes()).digest(), np.uint8),
             kind=vi.engine.sweep_kind)
    print(path, "kind", vi.engine.sweep_kind, "mean[0,0,:3]", vi.X_mean.numpy()[0, 0, :3])


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in ("mean", "covdiag", "covsha"):
        d = np.argwhere(A[k] != B[k])
        if len(d):
            ok = False
            print(f"{k}: {len(d)} entries differ, max |diff| {np.abs(A[k] - B[k]).max():.3e}, first {d[:5].tolist()}")
    print("BIT-EQUAL" if ok else "DIFFERENT", "kinds", int(A["kind"]), int(B["kind"]))
    return ok


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(*sys.argv[2:])
    else:
        sys.exit(0 if cmp(sys.argv[2], sys.argv[3]) else 1)
