"""Parity margins of one library build against the fp64 oracle (GPU box):
prints, per case, the GPU mean error, the fp32-oracle error (the tests'
allowance) and the covariance error, without asserting.

    AME_LIB_PATH=lib.so python tools/parity_margin.py n,T,r,method,lr[,kind] ...
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import ame_oracle as O
    from ame_amd import TemporalAMEModel
    from test_gpu_large import _params, _vi
    dev = torch.device("cuda", 0)
    for spec in sys.argv[1:]:
        f = spec.split(",")
        n, T, r, method, lr = int(f[0]), int(f[1]), int(f[2]), f[3], float(f[4])
        opts = {"sweep_kernel": int(f[5])} if len(f) > 5 else {}
        m = TemporalAMEModel(n, T, r, seed=7)
        m.generate_data_fast(seed=11)
        vi = _vi(m, method, lr, dev, **opts)
        Xm = vi.X_mean.numpy().astype(np.float64).copy()
        Xc = vi.X_cov.numpy().astype(np.float64).copy()
        Xm32, Xc32 = vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()
        O.fit(m.Y.numpy().astype(np.float64), Xm, Xc, _params(m), method, lr, 2, 0.0)
        O.fit(m.Y.numpy(), Xm32, Xc32, _params(m, np.float32), method, lr, 2, 0.0)
        fp32_err = np.abs(Xm32.astype(np.float64) - Xm).max()
        vi.fit(max_iter=2, tolerance=0.0, verbose=False)
        err = np.abs(vi.X_mean.numpy() - Xm).max()
        cerr = np.abs(vi.X_cov.numpy() - Xc).max()
        print(f"{spec:28s} kind {vi.engine.sweep_kind:2d}  mean err {err:.3e}  fp32-oracle err {fp32_err:.3e}"
              f"  ratio {err / fp32_err:.2f}  cov err {cerr:.3e}", flush=True)


if __name__ == "__main__":
    main()
