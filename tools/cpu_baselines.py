"""CPU baselines in full (verdict r02 item 7): one whole fit()
iteration of each CPU restatement, timed on this host, no extrapolation.

    python tools/cpu_baselines.py [--configs 1,2,3] [--threads 1,4,16] > out.jsonl

* loop restatement (oracle/ame_loop_oracle.py: the reference's per-dyad /
  per-pair torch op sequence, one core): configs 1 and 2 in full -- the
  sweep over every (node, t), the loglik over every pair and t, the MSE;
* vectorised numpy restatement (oracle/ame_oracle.py, the fair CPU baseline):
  one full iteration at configs 1-3 for each BLAS thread count given.

Data: the build's reference-stream generator at configs 1-2 (the reference's
own Y), the vectorised generator at config 3; SMF-good, lr = 0.01, state after
the VI initialisation (the time of one iteration does not depend on the
state).  Each line names the host (os.cpu_count(), CPU model) and the threads.
On the GPU box the process's CPU share is 16 cores (the harness sets
OMP_NUM_THREADS=16 and asks worker pools to stay within it), so 16 is the
largest thread count run there.  TEST / BASELINE INFRASTRUCTURE ONLY.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

CONFIGS = {1: (15, 10, 2), 2: (256, 64, 8), 3: (1024, 128, 16)}


def host():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"host_cpus": os.cpu_count(), "cpu_model": model}


def setup(cfg):
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    n, T, r = CONFIGS[cfg]
    m = TemporalAMEModel(n, T, r, seed=42)
    if cfg <= 2:
        m.generate_data()
    else:
        m.generate_data_fast(seed=42)
    vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=0.01)
    params = {k: getattr(m, k).numpy().astype(np.float32)
              for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")}
    return m, vi, params


def loop_iteration(m, vi, params):
    import ame_loop_oracle as LO
    Y = m.Y.float()
    Xm, Xc = vi.X_mean.clone(), vi.X_cov.clone()
    n, T = m.n, m.T
    t0 = time.perf_counter()
    for i in range(n):
        LO.update_node_loop(Y, Xm, Xc, params, i, "good", 0.01)
    t_sweep = time.perf_counter() - t0
    print(f"loop sweep n={n} T={T}: {t_sweep:.1f} s", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for t in range(T):
        LO.loglik_pairs_loop(Y, Xm, Xc, params, "good", t)
        if t % 16 == 15:
            print(f"loop loglik t={t}", file=sys.stderr, flush=True)
    t_ll = time.perf_counter() - t0
    # priors + entropy: per-(node, t) d x d work in the reference too, taken from
    # the vectorised restatement (a few % of the loop iteration)
    import ame_oracle as O
    Xm64 = Xm.numpy().astype(np.float32)
    Xc64 = Xc.numpy().astype(np.float32)
    t0 = time.perf_counter()
    O.log_prior_initial(Xm64, Xc64, params)
    O.log_prior_transitions(Xm64, Xc64, params)
    O.entropy(Xc64)
    t_pe = time.perf_counter() - t0
    t0 = time.perf_counter()
    m.compute_temporal_reconstruction_error(Xm)
    t_rec = time.perf_counter() - t0
    return t_sweep, t_ll + t_pe, t_rec


def numpy_iteration(m, vi, params):
    import ame_oracle as O
    Y = m.Y.numpy().astype(np.float32)
    Xm = vi.X_mean.numpy().astype(np.float32).copy()
    Xc = vi.X_cov.numpy().astype(np.float32).copy()
    t0 = time.perf_counter()
    O.sweep(Y, Xm, Xc, params, "good", 0.01)
    t_sweep = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.elbo(Y, Xm, Xc, params, "good")
    t_elbo = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.recon_error(Y, Xm)
    t_rec = time.perf_counter() - t0
    return t_sweep, t_elbo, t_rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3")
    ap.add_argument("--threads", default="1,16")
    ap.add_argument("--loop-configs", default="1,2")
    args = ap.parse_args()
    from threadpoolctl import threadpool_limits
    cfgs = [int(c) for c in args.configs.split(",") if c]
    loop_cfgs = [int(c) for c in args.loop_configs.split(",") if c]
    hinfo = host()
    for cfg in cfgs:
        m, vi, params = setup(cfg)
        n, T, r = CONFIGS[cfg]
        units = T * n * (n - 1) / 2.0
        base = {"config": cfg, "n": n, "T": T, "latent_dim": r, "d": 2 + 2 * r, "variant": "good",
                "units_per_iteration": units, **hinfo}
        if cfg in loop_cfgs:
            torch.set_num_threads(1)
            ts, tl, tr = loop_iteration(m, vi, params)
            it = ts + tl + tr
            print(json.dumps({**base, "kind": "loop_restatement", "threads": 1, "s_per_iteration": it,
                              "sweep_s": ts, "loglik_prior_entropy_s": tl, "recon_s": tr,
                              "units_per_s": units / it, "full_iteration": True}), flush=True)
        for th in [int(x) for x in args.threads.split(",") if x]:
            with threadpool_limits(limits=th):
                torch.set_num_threads(th)
                ts, te, tr = numpy_iteration(m, vi, params)
            it = ts + te + tr
            print(json.dumps({**base, "kind": "numpy_restatement", "threads": th, "s_per_iteration": it,
                              "sweep_s": ts, "elbo_s": te, "recon_s": tr,
                              "units_per_s": units / it, "full_iteration": True}), flush=True)


if __name__ == "__main__":
    main()
