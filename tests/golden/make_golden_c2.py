"""Config-2 golden fixture from the reference itself.

TEST INFRASTRUCTURE ONLY.  Runs in the build container, where the reference
(Alfieriek/Python-Temporal-AME-SVI) is mounted read-only at /root/reference.
BASELINE config 2 is n=256, T=64, latent_dim=8 (d=18), seed 42, lr=0.01.  Y is
33.5 MB, too large to commit, so the fixture holds its SHA-256 (fp32 bytes,
reference layout (n, n, T, 2)) and the GPU test regenerates it with
ame_amd's reference-stream generator (TemporalAMEModel.generate_data) and
checks the digest before comparing.  Per (method, dtype) run it stores the
ELBO / MSE trajectories of 2 fit() iterations, the ELBO split after each, and
sampled X_mean rows / X_cov blocks after each iteration.

The reference's X (the latent trajectories, 1.2 MB) IS committed: X comes from
small MKL matvecs whose rounding depends on the host CPU's MKL code path (the
GPU box's EPYC rounds differently from this Xeon), while Y given X is
reproducible anywhere (ame_amd's generator forms U V^T with the sequential-FMA
order MKL's sgemm uses here, and the noise stream exactly).

Usage (from the repo root; one process per run, ~10 min each)::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c2.py good f32
    ...
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c2.py --x     # X only
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c2.py --merge

Reference call sites (file:line under /root/reference):
  * TemporalAMEModel.__init__ / generate_data   src/models/temporal_ame.py:93-220
  * TemporalAMEStructuredMFVI / NaiveMFVI init  src/inference/structured_mf.py:58-113, naive_mf.py:71-87
  * BaseVariationalInference.fit                src/inference/base.py:127-208
  * ELBO split                                   src/inference/structured_mf.py:115-209
"""
import hashlib
import os
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
PARTS = os.path.join(OUT, "_c2_parts")

N, T, R, LR, ITERS = 256, 64, 8, 0.01, 2
NODES = [0, 1, 2, 3, 17, 64, 127, 128, 191, 200, 254, 255]
COV_IT = [(0, 0), (0, 63), (1, 1), (127, 31), (128, 32), (255, 0), (255, 63)]


def sha(a):
    import numpy as np
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run(method, prec):
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import numpy as np
    import torch
    torch.set_num_threads(1)
    from src.models import TemporalAMEModel
    from src.inference import TemporalAMEStructuredMFVI, TemporalAMENaiveMFVI
    sys.path.insert(0, OUT)
    from make_golden import elbo_split, to_f64

    m = TemporalAMEModel(n_nodes=N, n_time=T, latent_dim=R, ar_coefficient=0.8,
                         rho_dyadic=0.5, seed=42)
    Y, X = m.generate_data(return_latents=True)
    rec = {"Y_sha256": np.array(sha(Y.numpy())), "X_sha256": np.array(sha(X.numpy())),
           "Y_rows": Y[NODES].numpy().copy()[:, :8]}
    if method == "naive":
        vi = TemporalAMENaiveMFVI(m, learning_rate=LR)
    else:
        vi = TemporalAMEStructuredMFVI(m, factorization=method, learning_rate=LR)
    rec["init_mean_sha256"] = np.array(sha(vi.X_mean.numpy()))
    rec["init_cov_sha256"] = np.array(sha(vi.X_cov.numpy()))
    prev = torch.get_default_dtype()
    if prec == "f64":
        to_f64(m, vi)
        torch.set_default_dtype(torch.float64)
    try:
        splits = []
        for it in range(1, ITERS + 1):
            vi.fit(max_iter=1, tolerance=0.0, verbose=False)
            splits.append(elbo_split(vi))
            rec[f"mean_rows_{it}"] = vi.X_mean[NODES].double().numpy().copy()
            rec[f"cov_blocks_{it}"] = np.stack(
                [vi.X_cov[i, t].double().numpy() for i, t in COV_IT])
        rec["elbo"] = np.array([float(e) for e in vi.history["elbo"]], dtype=np.float64)
        rec["recon"] = np.array(vi.history["reconstruction_error"], dtype=np.float64)
        rec["elbo_split"] = np.stack(splits)
    finally:
        torch.set_default_dtype(prev)
    os.makedirs(PARTS, exist_ok=True)
    np.savez(os.path.join(PARTS, f"{method}_{prec}.npz"), **rec)
    print(f"{method} {prec}: elbo {rec['elbo']} recon {rec['recon']}", flush=True)


def save_x():
    """The reference's latent trajectories X (generate_data), for the GPU box."""
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import numpy as np
    import torch
    torch.set_num_threads(1)
    from src.models import TemporalAMEModel
    m = TemporalAMEModel(n_nodes=N, n_time=T, latent_dim=R, ar_coefficient=0.8,
                         rho_dyadic=0.5, seed=42)
    Y, X = m.generate_data(return_latents=True)
    os.makedirs(PARTS, exist_ok=True)
    np.savez(os.path.join(PARTS, "X.npz"), X=X.numpy(), X_sha256=np.array(sha(X.numpy())),
             Y_sha256=np.array(sha(Y.numpy())))


def merge():
    import numpy as np
    out = {"nodes": np.array(NODES, dtype=np.int64), "cov_it": np.array(COV_IT, dtype=np.int64),
           "n": np.int64(N), "T": np.int64(T), "r": np.int64(R), "lr": np.float64(LR)}
    shas = set()
    for f in sorted(os.listdir(PARTS)):
        if not f.endswith(".npz"):
            continue
        if f == "X.npz":
            zx = np.load(os.path.join(PARTS, f))
            out["X_true"] = zx["X"]
            shas.add((str(zx["Y_sha256"]), str(zx["X_sha256"])))
            continue
        key = f[:-4]
        z = np.load(os.path.join(PARTS, f))
        shas.add((str(z["Y_sha256"]), str(z["X_sha256"])))
        out["Y_sha256"], out["X_sha256"] = z["Y_sha256"], z["X_sha256"]
        out["Y_rows"] = z["Y_rows"]
        for k in z.files:
            if k not in ("Y_sha256", "X_sha256", "Y_rows"):
                out[f"{key}__{k}"] = z[k]
    assert len(shas) == 1, shas
    path = os.path.join(OUT, "c2_reference.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


if __name__ == "__main__":
    if sys.argv[1:] == ["--merge"]:
        merge()
    elif sys.argv[1:] == ["--x"]:
        save_x()
    else:
        run(sys.argv[1], sys.argv[2])
