#!/usr/bin/env python
"""Benchmark: dyad-timestep ELBO updates/s of the temporal-AME SMF VI loop on MI355X.

One "step" = one fit() iteration of TemporalAMEStructuredMFVI (reference
base.py:170-181): Gauss-Seidel sweep + covariance update + ELBO + MSE, over the
synthetic BASELINE config 3 workload (n=1024 nodes, latent_dim=16 -> d=34,
T=128 time steps per GPU; weak scaling T_total = 128 * N, time-sharded).
Units per step = T_total * n(n-1)/2 (the unordered dyad-timesteps the ELBO sums).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  Inputs are resident in HBM before timing; the
timed region is K full fit() iterations bracketed by barrier + synchronize,
max over ranks.  `roofline` is for the dominant kernel, timed with HIP events
on the stream it runs on; `cpu_baseline` times the numpy oracle
(oracle/ame_oracle.py) on a bounded sample of the same workload on this host.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "dyad-timestep ELBO updates/sec at n=1024,T=128,d=16; 1/2/4/8-GPU scaling"
UNIT = "dyad-timestep ELBO updates/s"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def kernel_bytes(n, TL, d, swap_consistent=True):
    """Algorithmic HBM bytes per launch."""
    y_full = 8.0 * n * (n - 1) * TL
    return {
        # Y row of every ordered dyad + old means read + new means written
        # + old covariance read + damped covariance written
        "sweep": y_full + 8.0 * n * TL * d + 8.0 * n * TL * d * d,
        # each covariance read once
        "cov": 4.0 * n * TL * d * d,
        # Y (upper triangle if swap-consistent) + means
        "elbo": (y_full / 2 if swap_consistent else y_full) + 4.0 * n * TL * d,
        # the pair kernel alone: the same Y bytes + means
        "pairs": (y_full / 2 if swap_consistent else y_full) + 4.0 * n * TL * d,
    }


def _host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:  # pragma: no cover
        pass
    return {"host_cpus": os.cpu_count(), "cpu_model": model}


def cpu_baseline(model, vi, n, T, d, budget_s=24.0):
    """Time the CPU restatements (fp32, the reference's dtype) on bounded
    samples of the same iteration and extrapolate to one full iteration.

    * main value: the vectorised numpy oracle (oracle/ame_oracle.py; BLAS
      threads = the threads numpy uses on this host), SURVEY.md §8d(ii);
    * ``loop_restatement``: oracle/ame_loop_oracle.py, the reference's cost
      model (one small torch op sequence per ordered dyad / unordered pair,
      structured_mf.py:130-148, :303-324), SURVEY.md §8d(i).
    """
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ame_oracle as O
    import ame_loop_oracle as LO
    try:
        from threadpoolctl import threadpool_info
        threads = max([p.get("num_threads", 1) for p in threadpool_info()] + [1])
    except Exception:  # pragma: no cover
        threads = 1
    Y = model.Y.detach().cpu().numpy().astype(np.float32)
    Xm = vi.X_mean.numpy().astype(np.float32).copy()
    Xc = vi.X_cov.numpy().astype(np.float32).copy()
    params = {k: getattr(model, k).detach().cpu().numpy().astype(np.float32)
              for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")}
    consts = O.prior_terms(params, T, np.float32)
    # --- vectorised oracle: a block of nodes of the sweep ---
    t0 = time.perf_counter()
    O.update_node(Y, Xm, Xc, params, 0, "good", 0.01, consts)
    per_node = time.perf_counter() - t0
    k = int(max(1, min(n - 1, (0.6 * budget_s) / max(per_node, 1e-6))))
    t0 = time.perf_counter()
    for i in range(1, 1 + k):
        O.update_node(Y, Xm, Xc, params, i, "good", 0.01, consts)
    sweep_est = (time.perf_counter() - t0) / k * n
    # loglik + MSE on a set of whole slices
    t0 = time.perf_counter()
    O.expected_loglik(Y, Xm, Xc, params, "good", ts=range(1))
    per_slice = time.perf_counter() - t0
    m = int(max(1, min(T, (0.25 * budget_s) / max(2.0 * per_slice, 1e-6))))
    t0 = time.perf_counter()
    O.expected_loglik(Y, Xm, Xc, params, "good", ts=range(m))
    t_ll = (time.perf_counter() - t0) / m * T
    t0 = time.perf_counter()
    off = ~np.eye(n, dtype=bool)
    for t in range(m):
        mu = O.compute_mean(Xm[:, t].astype(np.float64), (d - 2) // 2)
        float((((Y[:, :, t] - mu) ** 2)[off]).sum())
    t_rec = (time.perf_counter() - t0) / m * T
    kn = min(n, 64)
    t0 = time.perf_counter()
    O.entropy(Xc[:kn])
    O.log_prior_transitions(Xm[:kn], Xc[:kn], params)
    O.log_prior_initial(Xm[:kn], Xc[:kn], params)
    t_node_terms = (time.perf_counter() - t0) / kn * n
    it_est = sweep_est + t_ll + t_rec + t_node_terms
    units = T * n * (n - 1) / 2.0
    # --- loop-structured restatement: exact-size sample of update steps and pairs ---
    Yt = torch.from_numpy(Y)
    Xm_t, Xc_t = torch.from_numpy(Xm), torch.from_numpy(Xc)
    lb = 0.15 * budget_s
    t0 = time.perf_counter()
    LO.update_node_loop(Yt, Xm_t, Xc_t, params, n - 1, "good", 0.01, ts=range(1))
    per_step = time.perf_counter() - t0
    ns = int(max(1, min(T - 1, lb / max(per_step, 1e-6))))
    t0 = time.perf_counter()
    LO.update_node_loop(Yt, Xm_t, Xc_t, params, n - 1, "good", 0.01, ts=range(1, 1 + ns))
    per_step = (time.perf_counter() - t0) / ns
    rng = np.random.default_rng(0)
    npairs = 2000
    t0 = time.perf_counter()
    sample = [(int(a), int(b)) for a, b in (sorted(rng.choice(n, 2, replace=False))
                                            for _ in range(npairs))]
    LO.loglik_pairs_loop(Yt, Xm_t, Xc_t, params, "good", 0, pairs=sample[:200])
    per_pair = (time.perf_counter() - t0) / 200
    npairs = int(max(200, min(200000, lb / max(per_pair, 1e-9))))
    sample = [(int(a), int(b)) for a, b in (sorted(rng.choice(n, 2, replace=False))
                                            for _ in range(npairs))]
    t0 = time.perf_counter()
    LO.loglik_pairs_loop(Yt, Xm_t, Xc_t, params, "good", 0, pairs=sample)
    per_pair = (time.perf_counter() - t0) / npairs
    loop_it = per_step * n * T + per_pair * units + t_rec + t_node_terms
    return {
        "value": units / it_est, "unit": UNIT, "cores": int(threads), "kind": "port",
        "sample": (f"numpy oracle (oracle/ame_oracle.py) fp32, {threads} BLAS threads: "
                   f"update_node for {k + 1} of {n} nodes x {T} slices, loglik+MSE for {m} of "
                   f"{T} slices, entropy/prior terms for {kn} nodes; extrapolated linearly to "
                   f"one full iteration (est. {it_est:.1f} s/iteration)"),
        **_host_info(),
        "loop_restatement": {
            "value": units / loop_it, "unit": UNIT, "cores": 1, "kind": "port",
            "sample": (f"oracle/ame_loop_oracle.py (reference cost model: a torch op sequence "
                       f"per ordered dyad / unordered pair, fp32): {ns} (node, t) update steps "
                       f"at n={n} ({per_step * 1e3:.1f} ms each), {npairs} loglik pairs "
                       f"({per_pair * 1e6:.1f} us each); extrapolated to one iteration "
                       f"(est. {loop_it / 3600:.2f} h/iteration)"),
        },
    }


def isolated_ms(eng, reps=5):
    """Average ms of the covariance-terms and ELBO launches alone on the GPU
    (no sweep beside them), HIP events recorded on the stream they run on."""
    eng.events.clear()
    eng.timing = True
    torch.cuda.synchronize(eng.dev)
    for _ in range(reps):
        eng.refresh_cov_terms()
        eng.launch_elbo()
        torch.cuda.synchronize(eng.dev)
    ms, _ = eng.kernel_ms()
    # the pair kernel alone (diagnostic entry point ame_elbo_pairs_diag)
    eng.events.clear()
    for _ in range(reps):
        eng.launch_elbo(pairs_only=True)
        torch.cuda.synchronize(eng.dev)
    ms["pairs"] = eng.kernel_ms()[0].get("pairs")
    eng.timing = False
    eng.invalidate()
    return ms


def load_pmc(tag):
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(path):
        return None
    try:
        z = json.load(open(path))
        if z.get("config_tag") != tag:
            return None
        return z
    except Exception:
        return None


def main():
    # stdout carries exactly one JSON line: anything a library prints there
    # (RCCL's version banner at communicator creation, ...) goes to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--t-per-gpu", type=int, default=128)
    ap.add_argument("--latent-dim", type=int, default=16)
    ap.add_argument("--variant", default="good", choices=["good", "bad", "naive"])
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=24.0)
    ap.add_argument("--force-dist", action="store_true",
                    help="use the process group (nccl) and the time-sharded path even at world size 1 "
                         "(checks RCCL initialisation on a one-GPU box)")
    args = ap.parse_args()

    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE",
              file=sys.stderr)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local_rank % max(ndev, 1))
    torch.cuda.set_device(dev)
    use_dist = world > 1 or args.force_dist
    if use_dist:
        dist.init_process_group("nccl", device_id=dev)

    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI

    n, r = args.n, args.latent_dim
    d = 2 + 2 * r
    T_total = args.t_per_gpu * world
    model = TemporalAMEModel(n, T_total, r, seed=42)
    model.generate_data_fast(device=dev)
    if args.variant == "naive":
        vi = TemporalAMENaiveMFVI(model, learning_rate=args.lr, device=dev,
                                  distributed=use_dist)
    else:
        vi = TemporalAMEStructuredMFVI(model, factorization=args.variant, learning_rate=args.lr,
                                       device=dev, distributed=use_dist)
    if args.warmup > 0:
        vi.fit(max_iter=args.warmup, tolerance=0.0, verbose=False)
    eng = vi.engine
    eng.timing = True
    eng.events.clear()

    def barrier():
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize(dev)

    barrier()
    t0 = time.perf_counter()
    hist = vi.fit(max_iter=args.steps, tolerance=0.0, verbose=False)
    barrier()
    dt = time.perf_counter() - t0
    if use_dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    kms, kcount = eng.kernel_ms()
    TL = eng.shard.T_local
    kb = kernel_bytes(n, TL, d, eng.swap_consistent)
    units_per_step = T_total * n * (n - 1) / 2.0
    value = units_per_step * args.steps / dt
    ms_step = dt / args.steps * 1e3
    b_iter = 8.0 * n * (n - 1) * T_total + 4.0 * n * (n - 1) * T_total \
        + 12.0 * n * T_total * d * d + 16.0 * n * T_total * d
    tag = f"n{n}_T{args.t_per_gpu}_r{r}_{args.variant}"
    pmc = (load_pmc(tag) or {}).get("kernels", {})
    # cov / elbo launches once more, alone on the GPU (after the timed region)
    iso = isolated_ms(eng)
    pipelined = bool(getattr(eng, "pipelined", False))
    kernels = {}
    for name, ms, how in (
            ("sweep", ms_step, "per-iteration time (one sweep retires per fit() iteration; "
                               "pipelined launches overlap, so a launch's own duration is not "
                               "a per-sweep figure)"),
            ("cov", iso.get("cov"), "isolated launch, HIP events on its stream"),
            ("elbo", iso.get("elbo"), "isolated launch (pair + node + final kernels), HIP "
                                      "events on its stream"),
            ("pairs", iso.get("pairs"), "the ELBO pair kernel alone (ame_pairs2_kernel, MFMA), "
                                        "isolated launch, HIP events on its stream")):
        ent = {"alg_bytes": kb[name], "ms": ms, "timing": how,
               "launch_ms_in_fit": kms.get(name)}
        if ms:
            ach = kb[name] / (ms * 1e-3) / 1e9
            ent.update(achieved_GBs=ach, frac=ach / HBM_PEAK_GBS)
        pk = pmc.get({"elbo": "pairs"}.get(name, name))   # elbo: its dominant (pair) kernel
        if pk:
            ent["traffic"] = pk.get("hbm_bytes_per_launch")
            ent["traffic_kernel"] = pk.get("kernel")
            if ent["traffic"]:
                alg = kb[name] if name != "elbo" else pk.get("alg_bytes", kb[name])
                ent["traffic_over_alg"] = ent["traffic"] / alg
        kernels[name] = ent
    sw = kernels["sweep"]

    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(model, vi, n, T_total, d, budget_s=args.cpu_budget)
        elbo_last = float(hist["elbo"][-1])
        shape = (n, args.t_per_gpu, r)
        named = {(1024, 128, 16): "BASELINE config 3 shape per GPU",
                 (256, 64, 8): "BASELINE config 2 shape per GPU",
                 (1024, 64, 16): "BASELINE config 4 per-rank shape (T=512 over 8 GPUs)",
                 (4096, 32, 32): "BASELINE config 5 per-rank shape (T=256 over 8 GPUs)"}
        label = named.get(shape, "custom shape")
        out = {
            "metric": METRIC, "value": value, "unit": UNIT, "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic",
            "config": {
                "workload": (f"{label}: n_nodes={n}, n_time={args.t_per_gpu}/GPU "
                             f"(T_total={T_total}), latent_dim={r} (d={d}), "
                             f"SMF-{args.variant} fit iteration, lr={args.lr}"),
                "n_nodes": n, "n_time_total": T_total, "latent_dim": r, "d": d,
                "variant": args.variant, "parallelism": f"time-sharded x{world}",
                "sweep_kind": int(vi.engine.sweep_kind),
            },
            "roofline": {"bound": "hbm", "kernel": "sweep", "achieved": sw["achieved_GBs"],
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": sw["frac"],
                         "traffic": sw.get("traffic"),
                         "note": ("achieved = the sweep's algorithmic bytes per launch "
                                  "(DESIGN.md §4) / ms_per_step: one sweep retires per "
                                  "iteration" + ("; launches are pipelined" if pipelined else "")
                                  + ". The sweep is latency-bound: n dependent node steps "
                                  "per slice")},
            "kernels": kernels,
            "schedule": {"pipelined": pipelined,
                         "sweeps_queued_ahead": int(getattr(eng, "spec_depth", 1))},
            "iteration_roofline_frac": b_iter / (dt / args.steps) / (world * HBM_PEAK_GBS * 1e9),
            "cpu_baseline": cpu,
            "elbo_last": elbo_last,
            "mse_last": float(hist["reconstruction_error"][-1]),
        }
        print(json.dumps(out), file=json_out, flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
