"""Covariance symmetry check (GPU box): fits repeated per engine setting,
printing how many entries differ from their mirror and by how much.
    python tools/symcheck.py n,T,r variant kind reps"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))


def main():
    import torch
    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    n, T, r = (int(x) for x in sys.argv[1].split(","))
    variant, kind, reps = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    dev = torch.device("cuda", 0)
    for pipe in (True, False):
        for spec in (True, False):
            for rep in range(reps):
                m = TemporalAMEModel(n, T, r, seed=2)
                m.generate_data_fast(seed=3)
                opts = {"sweep_kernel": kind, "pipeline": pipe, "speculate": spec}
                if variant == "naive":
                    vi = TemporalAMENaiveMFVI(m, learning_rate=0.7, device=dev, engine_options=opts)
                else:
                    vi = TemporalAMEStructuredMFVI(m, factorization=variant, learning_rate=0.7, device=dev,
                                                   engine_options=opts)
                C0 = vi.X_cov.numpy().copy()
                a0 = np.count_nonzero(C0 != np.swapaxes(C0, -1, -2))
                vi.fit(max_iter=2, tolerance=0.0, verbose=False)
                C = vi.X_cov.numpy()
                dif = np.abs(C - np.swapaxes(C, -1, -2))
                bad = np.argwhere(dif > 0)
                print(f"pipe={pipe} spec={spec} rep={rep} kind={vi.engine.sweep_kind} pipelined={vi.engine.pipelined} "
                      f"init asym {a0}  asym {len(bad)} max {dif.max():.3e} first {bad[:3].tolist()}", flush=True)


if __name__ == "__main__":
    main()
