"""Phase timeline of the MFMA covariance-terms kernel (AME_COV_STAMPS build):

    AME_LIB_PATH=tools/_lib/libame_amd_covst32.so python tools/cov_stamps.py [n T r]

Runs ame_cov once on random SPD covariances of the shape (tools/cov_ab.py's
data) and prints, for wave 0 of block 0, the mean s_memtime ticks of each
phase over its covariances 2..15: loads + traces, Schur MFMAs, tile columns
0..3 of the blocked LDL^T, log / reduction / store."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402


def main():
    n, T, r = (int(x) for x in (sys.argv[1:4] or (4096, 32, 32)))
    import torch
    from ame_amd import _lib
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    d = 2 + 2 * r
    g = torch.Generator(device=dev).manual_seed(1)
    cov = torch.empty(T * n, d, d, device=dev)
    for s in range(0, T * n, 8192):
        X = torch.randn(min(8192, T * n - s), d, 2 * d, device=dev, generator=g)
        cov[s:s + X.shape[0]] = X @ X.transpose(1, 2) / (2 * d) + 0.25 * torch.eye(d, device=dev)
    consts = torch.zeros(5, d, d, dtype=torch.float64, device=dev)
    consts[0] = torch.eye(d, dtype=torch.float64) * 0.5
    consts[1] = torch.eye(d, dtype=torch.float64) * 2.0
    out = torch.zeros(T * n * 4, dtype=torch.float64, device=dev)
    dims = _lib.ame_dims(n, r, T, 1, T + 1, 0)   # no slice 0: one launch
    args = _lib.ame_cov_args(cov=cov.data_ptr(), consts=consts.data_ptr(), cov_terms=out.data_ptr())
    _lib.check(L.ame_cov(ctypes.byref(dims), ctypes.byref(args), None), "ame_cov")
    torch.cuda.synchronize()
    st = (ctypes.c_ulonglong * (16 * 8))()
    assert L.ame_debug_read_cov_stamps(st) == 0
    a = np.array(st[:], dtype=np.float64).reshape(16, 8)
    names = ["loads + traces", "Schur MFMAs", "tile column 0", "tile column 1", "tile column 2",
             "tile column 3", "log + sums + store"]
    dt = np.diff(a[2:16], axis=1)
    per = a[3:16, 0] - a[2:15, 0]
    print(f"n={n} T={T} r={r}: covariance period {per.mean():.0f} ticks (wave 0 of block 0, covariances 2..15)")
    for k, nm in enumerate(names):
        print(f"  {nm:22s} {dt[:, k].mean():8.0f}")


if __name__ == "__main__":
    main()
