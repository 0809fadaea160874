"""Worker (kind 22) vs single-workgroup v2 (kind 20) vs the fp64 oracle on one case."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-temporal-ame-svi_amd"), os.path.join(ROOT, "oracle")]
import torch
import ame_oracle as O
from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI, TemporalAMENaiveMFVI
PK = ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")
dev = torch.device("cuda", 0)
for (n, T, r, meth, lr, it) in [(9, 1, 32, "bad", 0.4, 2), (9, 1, 32, "bad", 0.4, 1), (9, 1, 32, "good", 0.4, 2),
                                (12, 1, 32, "bad", 0.4, 2), (40, 1, 32, "good", 0.01, 2)]:
    m = TemporalAMEModel(n, T, r, seed=7); m.generate_data_fast(seed=11)
    res = {}
    for mode in ("0", "1"):
        os.environ["AME_SWEEP_NOWORKERS"] = mode
        vi = (TemporalAMENaiveMFVI(m, learning_rate=lr, device=dev) if meth == "naive" else
              TemporalAMEStructuredMFVI(m, factorization=meth, learning_rate=lr, device=dev))
        Xm = vi.X_mean.numpy().astype(np.float64).copy(); Xc = vi.X_cov.numpy().astype(np.float64).copy()
        p = {k: getattr(m, k).numpy().astype(np.float64) for k in PK}
        O.fit(m.Y.numpy().astype(np.float64), Xm, Xc, p, meth, lr, it, 0.0)
        vi.fit(max_iter=it, tolerance=0.0, verbose=False)
        gm, gc = vi.X_mean.numpy(), vi.X_cov.numpy()
        res[mode] = (gm.copy(), gc.copy())
        dm = np.abs(gm - Xm); dc = np.abs(gc - Xc)
        print(f"n={n} T={T} {meth} lr={lr} it={it} kind={vi.engine.sweep_kind}: mean err {dm.max():.2e} "
              f"(node {np.unravel_index(dm.argmax(), dm.shape)[0]}), cov err {dc.max():.2e} "
              f"(node {np.unravel_index(dc.argmax(), dc.shape)[0]})", flush=True)
    print("   worker vs v2: mean", np.abs(res["0"][0] - res["1"][0]).max(), "cov", np.abs(res["0"][1] - res["1"][1]).max())
