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


def _committed_full_iteration(n, T, r):
    """Full-iteration CPU measurements of the direct numpy restatement committed
    by tools/cpu_baselines.py (profiles/r03_cpu_baselines.jsonl) for this shape."""
    path = os.path.join(ROOT, "profiles", "r03_cpu_baselines.jsonl")
    out = []
    if os.path.exists(path):
        for line in open(path):
            try:
                z = json.loads(line)
            except ValueError:
                continue
            if (z.get("n"), z.get("T"), z.get("latent_dim")) == (n, T, r) and z.get("full_iteration"):
                out.append({k: z.get(k) for k in ("kind", "threads", "s_per_iteration", "units_per_s",
                                                  "cpu_model")})
    return out or None


def cpu_baseline(model, vi, n, T, d, budget_s=40.0):
    """CPU baselines on this host, fp64 / fp32 restatements of the same iteration
    (SURVEY.md §8d), timed after the GPU's timed region:

    * main value: the vectorised numpy oracle in its statistics form
      (oracle/ame_oracle.py sweep_stats + elbo_recon_fast) in fp32, the
      reference's dtype, BLAS threads as numpy uses them: ONE FULL ITERATION
      measured, not extrapolated, when the sweep's estimate fits `budget_s`
      (config 3: it does); otherwise the sweep is timed on a node prefix and
      extrapolated (said in `sample`); the same in fp64 (the parity oracle)
      beside it as ``fp64_statistics_form``;
    * ``direct_restatement``: the per-step restatement (update_node: P_obs / h_obs
      summed over all other nodes at every step, as the reference does) on a
      node sample, extrapolated; plus its committed full-iteration figures
      for this shape, if any (tools/cpu_baselines.py);
    * ``loop_restatement``: oracle/ame_loop_oracle.py, the reference's cost model
      (one small torch op sequence per ordered dyad / unordered pair,
      structured_mf.py:130-148, :303-324), 1 core, on a sample, extrapolated.
    """
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ame_oracle as O
    import ame_loop_oracle as LO
    try:
        from threadpoolctl import threadpool_info
        threads = max([p.get("num_threads", 1) for p in threadpool_info()] + [1])
    except Exception:  # pragma: no cover
        threads = 1
    r = (d - 2) // 2
    Y = model.Y.detach().cpu().numpy().astype(np.float32)
    X32 = vi.X_mean.numpy().astype(np.float32).copy()
    C32 = vi.X_cov.numpy().astype(np.float32).copy()
    params = {k: getattr(model, k).detach().cpu().numpy().astype(np.float32)
              for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")}
    units = T * n * (n - 1) / 2.0

    def stats_iteration(dt):
        """One iteration of the statistics-form oracle in dtype dt: the full
        sweep when its estimate fits the budget (else a node prefix,
        extrapolated), then the ELBO / MSE."""
        Xm, Xc = X32.astype(dt), C32.astype(dt)
        k0 = min(n, 16)
        t0 = time.perf_counter()
        O.sweep_stats(Y, Xm, Xc, params, "good", 0.01, nodes=range(k0))
        t_head = time.perf_counter() - t0
        est = t_head / k0 * n
        if k0 < n and est <= budget_s:
            t0 = time.perf_counter()
            O.sweep_stats(Y, Xm, Xc, params, "good", 0.01, nodes=range(k0, n))
            t_sw = t_head + time.perf_counter() - t0
            sw = n
        else:
            t_sw, sw = est, k0
        mT = T if n * n * T <= (1 << 28) else max(1, (1 << 28) // (n * n))
        t0 = time.perf_counter()
        O.elbo_recon_fast(Y[:, :, :mT], Xm[:, :mT], Xc[:, :mT], params, "good", dtype=dt)
        t_el = (time.perf_counter() - t0) * T / mT
        return t_sw, sw, t_el, mT

    # --- statistics-form oracle: one full iteration, fp32 (the reference's
    # dtype) as the value, fp64 (the parity oracle) beside it ---
    t_sweep, swept, t_elbo, mT = stats_iteration(np.float32)
    it_s = t_sweep + t_elbo
    full = swept == n and mT == T
    t_sweep64, swept64, t_elbo64, mT64 = stats_iteration(np.float64)
    it64 = t_sweep64 + t_elbo64
    # --- direct restatement: a node sample of the sweep, extrapolated ---
    Xd, Cd = X32.copy(), C32.copy()
    consts = O.prior_terms(params, T, np.float32)
    t0 = time.perf_counter()
    O.update_node(Y, Xd, Cd, params, 0, "good", 0.01, consts)
    per_node = time.perf_counter() - t0
    kd = int(max(1, min(n - 1, (0.15 * budget_s) / max(per_node, 1e-6))))
    t0 = time.perf_counter()
    for i in range(1, 1 + kd):
        O.update_node(Y, Xd, Cd, params, i, "good", 0.01, consts)
    direct_sweep = (time.perf_counter() - t0) / kd * n
    direct_it = direct_sweep + t_elbo
    # --- loop-structured restatement: exact-size sample of update steps and pairs ---
    Yt = torch.from_numpy(Y)
    Xm_t, Xc_t = torch.from_numpy(X32.copy()), torch.from_numpy(C32.copy())
    lb = 0.08 * budget_s
    t0 = time.perf_counter()
    LO.update_node_loop(Yt, Xm_t, Xc_t, params, n - 1, "good", 0.01, ts=range(1))
    per_step = time.perf_counter() - t0
    ns = int(max(1, min(T - 1, lb / max(per_step, 1e-6))))
    t0 = time.perf_counter()
    LO.update_node_loop(Yt, Xm_t, Xc_t, params, n - 1, "good", 0.01, ts=range(1, 1 + ns))
    per_step = (time.perf_counter() - t0) / ns
    rng = np.random.default_rng(0)
    sample = [(int(a), int(b)) for a, b in (sorted(rng.choice(n, 2, replace=False))
                                            for _ in range(200))]
    t0 = time.perf_counter()
    LO.loglik_pairs_loop(Yt, Xm_t, Xc_t, params, "good", 0, pairs=sample)
    per_pair = (time.perf_counter() - t0) / 200
    npairs = int(max(200, min(200000, lb / max(per_pair, 1e-9))))
    sample = [(int(a), int(b)) for a, b in (sorted(rng.choice(n, 2, replace=False))
                                            for _ in range(npairs))]
    t0 = time.perf_counter()
    LO.loglik_pairs_loop(Yt, Xm_t, Xc_t, params, "good", 0, pairs=sample)
    per_pair = (time.perf_counter() - t0) / npairs
    loop_it = per_step * n * T + per_pair * units + t_elbo
    how = ("one full iteration measured (no extrapolation)" if full else
           f"sweep timed on {swept} of {n} nodes, loglik / MSE on {mT} of {T} slices, "
           "extrapolated linearly")
    return {
        "value": units / it_s, "unit": UNIT, "cores": int(threads), "kind": "port",
        "full_iteration": full, "s_per_iteration": it_s,
        "sample": (f"numpy oracle, statistics form (oracle/ame_oracle.py sweep_stats + "
                   f"elbo_recon_fast), fp32, {threads} BLAS threads: {how}; sweep {t_sweep:.1f} s "
                   f"+ ELBO / MSE {t_elbo:.1f} s = {it_s:.1f} s per iteration"),
        **_host_info(),
        "fp64_statistics_form": {
            "value": units / it64, "unit": UNIT, "cores": int(threads), "kind": "port",
            "s_per_iteration": it64, "full_iteration": swept64 == n and mT64 == T,
            "sample": f"the same in fp64 (the parity oracle): sweep {t_sweep64:.1f} s + ELBO / MSE "
                      f"{t_elbo64:.1f} s"},
        "direct_restatement": {
            "value": units / direct_it, "unit": UNIT, "cores": int(threads), "kind": "port",
            "sample": (f"oracle/ame_oracle.py update_node (P_obs / h_obs re-summed over all "
                       f"nodes at every step, as the reference), fp32: {kd + 1} of {n} nodes x "
                       f"{T} slices, extrapolated (sweep est. {direct_sweep:.1f} s) + the "
                       f"ELBO / MSE above"),
            "committed_full_iterations": _committed_full_iteration(n, T, r),
        },
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
    """The committed PMC summary (tools/pmc_summary.py) whose config_tag is this
    shape: profiles/pmc_latest.json (config 3) or profiles/pmc_latest_*.json."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_latest*.json"))):
        try:
            z = json.load(open(path))
        except Exception:
            continue
        if z.get("config_tag") == tag:
            z["_file"] = os.path.relpath(path, ROOT)
            return z
    return None


# node steps of wavefront lag per slice of the in-order GEMV-worker sweep (kind
# 22), measured directly: slice-to-slice start lag at step 256, median over the
# 31 hops of config 5's rank shape, 1.26-1.46 in nine stamped runs
# (s_memrealtime on every slice; profiles/r05_c5_lag_stamps.txt,
# r05_c5_prologue_stamps.txt), rounded up.  (Round 5 first used 3.0 from whole
# iteration times at T_local = 32 vs 1, profiles/r05_d_c5_fill.jsonl, which
# also carry the per-launch prologue and the per-step cost of a fuller chip.)
FILL_STEPS_KIND22 = 1.5


def scaling_model(n, T_total, world, depth, pipelined, fill=None):
    """DESIGN.md §5 queue-depth model: node steps per iteration at this world
    size, against one GPU's n (predicted weak-scaling efficiency = n / that).
    Pipelined: max(n + hop, (F (T_total - 1) + n + delta) / (1 + depth));
    in order: the fill F (T_total - 1) + n every iteration."""
    sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))
    from ame_amd.engine import ELBO_READ_STEPS, FILL_STEPS_PER_SLICE
    F = FILL_STEPS_PER_SLICE if fill is None else fill
    hop = world - 1          # about one node step per rank boundary
    fill_steps = F * (T_total - 1)
    if pipelined:
        steps = max(n + hop, (fill_steps + n + ELBO_READ_STEPS) / (1 + depth))
        one = max(n, (F * (T_total // world - 1) + n + ELBO_READ_STEPS) / (1 + depth))
    else:
        steps = fill_steps + n
        one = F * (T_total // world - 1) + n
    return {"node_steps_per_iteration": steps, "one_gpu_node_steps": one,
            "predicted_efficiency_vs_1gpu": one / steps, "spec_depth": depth,
            "fill_steps_per_slice": F}


def _lib_provenance():
    try:
        from ame_amd import _lib
        return _lib.provenance()
    except Exception as e:  # pragma: no cover
        return {"error": str(e)}


def secondary_config5(dev, steps=8, warmup=2):
    """BASELINE config 5's per-rank shape (n=4096, T_local=32, r=32, SMF-good,
    lr 0.01; the GEMV-worker sweep) on the same GPU after the main measurement,
    so the driver's record carries the largest configuration too.  Reported
    beside the metric, never as it.  Carries its own roofline (the sweep's
    algorithmic bytes per iteration, PMC traffic from the committed pass),
    per-kernel HIP-event times and the queue-depth scaling model at N = 8
    (T_total = 256)."""
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    try:
        n, TL, r = 4096, 32, 32
        d = 2 + 2 * r
        # the config-3 state stays resident (≈ 3 GB beside config 5's ≈ 9 GB)
        m5 = TemporalAMEModel(n, TL, r, seed=42)
        m5.generate_data_fast(device=dev)
        v5 = TemporalAMEStructuredMFVI(m5, factorization="good", learning_rate=0.01, device=dev)
        v5.fit(max_iter=warmup, tolerance=0.0, verbose=False)
        eng = v5.engine
        eng.timing = True
        eng.events.clear()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        v5.fit(max_iter=steps, tolerance=0.0, verbose=False)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        kms, _ = eng.kernel_ms()
        iso = isolated_ms(eng)
        ms = dt / steps * 1e3
        units = TL * n * (n - 1) / 2.0
        kb = kernel_bytes(n, TL, d, eng.swap_consistent)
        pmc_all = load_pmc(f"n{n}_T{TL}_r{r}_good") or {}
        pmc = pmc_all.get("kernels", {})
        kernels = {}
        for name, kms_v, how in (
                ("sweep", ms, "per-iteration time (in-order sweeps: one per iteration)"),
                ("cov", iso.get("cov"), "isolated launch, HIP events on its stream"),
                ("elbo", iso.get("elbo"), "isolated launch (pair + node + final kernels)"),
                ("pairs", iso.get("pairs"), "the ELBO pair kernel alone, isolated launch")):
            ent = {"alg_bytes": kb[name], "ms": kms_v, "timing": how,
                   "launch_ms_in_fit": kms.get(name)}
            if kms_v:
                ach = kb[name] / (kms_v * 1e-3) / 1e9
                ent.update(achieved_GBs=ach, frac=ach / HBM_PEAK_GBS)
            pk = pmc.get({"elbo": "pairs"}.get(name, name))
            if pk and pk.get("hbm_bytes_per_launch"):
                ent["traffic"] = pk["hbm_bytes_per_launch"]
                ent["traffic_over_alg"] = pk["hbm_bytes_per_launch"] / pk.get("alg_bytes", kb[name])
                ent["traffic_source"] = pmc_all.get("_file")
            kernels[name] = ent
        sw = kernels["sweep"]
        if kms.get("sweep"):
            sw["frac_per_launch"] = kb["sweep"] / (kms["sweep"] * 1e-3) / 1e9 / HBM_PEAK_GBS
        pipelined = bool(eng.pipelined)
        depth = int(getattr(eng, "spec_depth", 1))
        return {"config": "BASELINE config 5 per-rank shape: n_nodes=4096, n_time=32, latent_dim=32 "
                          "(d=66), SMF-good fit iteration, lr=0.01, one GPU",
                "ms_per_step": ms, "value": units / (ms * 1e-3), "unit": UNIT, "steps": steps,
                "warmup": warmup, "sweep_kind": int(eng.sweep_kind), "pipelined": pipelined,
                "roofline": {"bound": "hbm", "kernel": "sweep", "achieved": sw.get("achieved_GBs"),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": sw.get("frac"),
                             "traffic": sw.get("traffic"),
                             "traffic_over_alg": sw.get("traffic_over_alg"),
                             "note": "achieved = the sweep's algorithmic bytes per launch / "
                                     "ms_per_step; traffic from the committed PMC pass"},
                "kernels": kernels,
                "scaling_model": scaling_model(n, TL * 8, 8, depth, pipelined,
                                               fill=FILL_STEPS_KIND22 if not pipelined else None),
                "scaling_model_note": "config 5 time-sharded over 8 GPUs (T_total = 256): "
                                      "node steps per iteration at N = 8 vs one rank's 32 slices"}
    except Exception as e:   # never costs the main line
        return {"error": f"{type(e).__name__}: {e}"}


def sweep_alg_bytes(n, TL, d):
    return kernel_bytes(n, TL, d)["sweep"]


def config5_full(dev, steps=3, warmup=1, variants=("naive", "good", "bad"), opts=None):
    """BASELINE config 5's own workload on ONE GPU: n=4096, T=256, r=32 (d=66),
    Naive-MF vs SMF-good vs SMF-bad on the same synthetic Y
    (experiments/three_way_conparison.py:141-179).  The GEMV-worker sweep
    (kind 22) runs as 8 consecutive slice groups of 32 per iteration.  Per
    variant: `warmup` untimed fit() iterations, then `steps` timed ones
    (synchronize on both sides) with HIP events around every kernel launch."""
    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    n, T, r = 4096, 256, 32
    d = 2 + 2 * r
    m = TemporalAMEModel(n, T, r, seed=42)
    m.generate_data_fast(device=dev)
    units = T * n * (n - 1) / 2.0
    out = {"metric": "config 5 three-way fit() iteration time", "unit": "ms/iteration",
           "config": {"workload": "BASELINE config 5 on one GPU: n_nodes=4096, n_time=256, "
                                  "latent_dim=32 (d=66), Naive-MF / SMF-good / SMF-bad on one Y, "
                                  "lr=0.01", "n_nodes": n, "n_time": T, "latent_dim": r},
           "steps": steps, "warmup": warmup, "data": "synthetic", "dtype": "f32", "variants": {}}
    for method in variants:
        if method == "naive":
            vi = TemporalAMENaiveMFVI(m, learning_rate=0.01, device=dev, engine_options=opts)
        else:
            vi = TemporalAMEStructuredMFVI(m, factorization=method, learning_rate=0.01, device=dev,
                                           engine_options=opts)
        eng = vi.engine
        vi.fit(max_iter=warmup, tolerance=0.0, verbose=False)
        eng.timing = True
        eng.events.clear()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        h = vi.fit(max_iter=steps, tolerance=0.0, verbose=False)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        kms, kcount = eng.kernel_ms()
        ms = dt / steps * 1e3
        alg = sweep_alg_bytes(n, T, d)
        out["variants"][method] = {
            "ms_per_iteration": ms, "updates_per_s": units / (ms * 1e-3),
            "sweep_kind": int(eng.sweep_kind), "slice_groups": len(eng.groups),
            "pipelined": bool(eng.pipelined), "sweeps_queued_ahead": int(eng.spec_depth),
            "kernel_ms": kms, "kernel_launches": kcount,
            "sweep_roofline": {"alg_bytes": alg, "ms": kms.get("sweep"),
                               "frac": (alg / (kms["sweep"] * 1e-3) / 1e9 / HBM_PEAK_GBS)
                               if kms.get("sweep") else None,
                               "note": "algorithmic bytes of one full sweep (8 slice-group "
                                       "launches) / its HIP-event time"},
            "elbo_last": float(h["elbo"][-1]), "mse_last": float(h["reconstruction_error"][-1])}
        del vi, eng
        torch.cuda.empty_cache()
    return out


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
    ap.add_argument("--cpu-budget", type=float, default=40.0)
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the second, untimed-by-the-driver measurement of BASELINE "
                         "config 5's per-rank shape (N=1 default runs only)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="sweeps in order (profiling: per-dispatch counters without the "
                         "pipelined launches' waiting)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="process-group backend under torchrun (nccl = RCCL, the production "
                         "path; gloo rehearses the multi-rank bench with several ranks on one GPU, "
                         "where RCCL refuses two ranks per device)")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the process group (nccl) and the time-sharded path even at world size 1 "
                         "(checks RCCL initialisation on a one-GPU box)")
    ap.add_argument("--sweep-kernel", type=int, default=0,
                    help="sweep kernel request (include/ame_amd.h enum ame_sweep_kind_code; "
                         "0 = AUTO, the production choice)")
    ap.add_argument("--elbo-cus", type=int, default=0,
                    help="run the ELBO kernels on a CU-masked stream over this many CUs beside "
                         "the sweep (engine option elbo_cus; needs --sweep-kernel 22 or 24)")
    ap.add_argument("--elbo-first", choices=("auto", "on", "off"), default="auto",
                    help="queue each iteration's ELBO before the speculative next sweep (engine "
                         "option elbo_first; auto = the engine default, off)")
    ap.add_argument("--config5-full", action="store_true",
                    help="BASELINE config 5's own workload (n=4096, T=256, r=32) three-way on "
                         "this one GPU; prints its own JSON line instead of the metric")
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
    if args.config5_full:
        c5opts = {"sweep_kernel": args.sweep_kernel} if args.sweep_kernel else None
        if args.elbo_cus:
            c5opts = dict(c5opts or {}, elbo_cus=args.elbo_cus)
        if args.no_pipeline:
            c5opts = dict(c5opts or {}, pipeline=False)
        if args.elbo_first != "auto":
            c5opts = dict(c5opts or {}, elbo_first=args.elbo_first == "on")
        out = config5_full(dev, steps=args.steps if args.steps != 50 else 3,
                           warmup=args.warmup if args.warmup != 3 else 1, opts=c5opts)
        print(json.dumps(out), file=json_out, flush=True)
        return out
    if use_dist:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI

    n, r = args.n, args.latent_dim
    d = 2 + 2 * r
    T_total = args.t_per_gpu * world
    model = TemporalAMEModel(n, T_total, r, seed=42)
    model.generate_data_fast(device=dev)
    opts = {"pipeline": False} if args.no_pipeline else {}
    if args.sweep_kernel:
        opts["sweep_kernel"] = args.sweep_kernel
    if args.elbo_cus:
        opts["elbo_cus"] = args.elbo_cus
    if args.elbo_first != "auto":
        opts["elbo_first"] = args.elbo_first == "on"
    opts = opts or None
    if args.variant == "naive":
        vi = TemporalAMENaiveMFVI(model, learning_rate=args.lr, device=dev,
                                  distributed=use_dist, engine_options=opts)
    else:
        vi = TemporalAMEStructuredMFVI(model, factorization=args.variant, learning_rate=args.lr,
                                       device=dev, distributed=use_dist, engine_options=opts)
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
    # device-side cross-rank wait time (status words 11 / 12, microseconds summed
    # over sweeps; include/ame_amd.h): read before and after the timed region
    cw0 = eng.status[11:13].cpu().tolist()
    t0 = time.perf_counter()
    hist = vi.fit(max_iter=args.steps, tolerance=0.0, verbose=False)
    barrier()
    dt = time.perf_counter() - t0
    cw1 = eng.status[11:13].cpu().tolist()
    cross_ms = [((b - a) & 0xFFFFFFFF) / 1e3 / args.steps for a, b in zip(cw0, cw1)]
    per_rank_ms = [dt / args.steps * 1e3]
    per_rank_cross = [cross_ms]
    if use_dist:
        tt = torch.tensor([dt, cross_ms[0], cross_ms[1]], dtype=torch.float64,
                          device=dev if args.dist_backend == "nccl" else "cpu")
        allt = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(allt, tt)
        per_rank_ms = [float(x[0].item()) / args.steps * 1e3 for x in allt]
        per_rank_cross = [[float(x[1].item()), float(x[2].item())] for x in allt]
        tt = tt[:1].clone()
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
    pmc_all = load_pmc(tag) or {}
    pmc = pmc_all.get("kernels", {})
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
        if name == "sweep" and kms.get("sweep"):
            # the same bytes over the launch's own HIP-event duration (the rocprof
            # kernel-statistics basis): a pipelined launch's span includes waiting
            # for the previous sweep's slices, so this is the lower of the two
            ent["frac_per_launch"] = kb[name] / (kms["sweep"] * 1e-3) / 1e9 / HBM_PEAK_GBS
            ent["frac_basis"] = {"frac": "algorithmic bytes / ms_per_step (one sweep retires "
                                         "per iteration)",
                                 "frac_per_launch": "algorithmic bytes / launch_ms_in_fit "
                                                    "(HIP events around each launch)"}
        pk = pmc.get({"elbo": "pairs"}.get(name, name))   # elbo: its dominant (pair) kernel
        if pk:
            ent["traffic"] = pk.get("hbm_bytes_per_launch")
            ent["traffic_kernel"] = pk.get("kernel")
            ent["traffic_source"] = pmc_all.get("_file")
            if ent["traffic"]:
                alg = kb[name] if name != "elbo" else pk.get("alg_bytes", kb[name])
                ent["traffic_over_alg"] = ent["traffic"] / alg
            if name == "pairs" and pk.get("mfma_busy") is not None:
                ent["mfma_busy"] = pk["mfma_busy"]
                ent["mfma_method"] = pk.get("mfma_method")
        kernels[name] = ent
    sw = kernels["sweep"]

    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(model, vi, n, T_total, d, budget_s=args.cpu_budget)
        elbo_last = float(hist["elbo"][-1])
        shape = (n, args.t_per_gpu, r)
        secondary = None
        # the full default run only (tools pass --no-cpu-baseline: profiler passes
        # and A/B runs see the config-3 kernels alone)
        if (world == 1 and not args.no_secondary and not args.no_cpu_baseline
                and shape == (1024, 128, 16) and args.variant == "good"):
            secondary = secondary_config5(dev)
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
                **({"elbo_cus": args.elbo_cus} if args.elbo_cus else {}),
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
                         "sweeps_queued_ahead": int(getattr(eng, "spec_depth", 1)),
                         "elbo_first": bool(getattr(eng, "elbo_first", False))},
            "per_rank_ms_per_step": per_rank_ms,
            "per_rank_cross_wait_ms_per_step": {
                "halo": [c[0] for c in per_rank_cross], "back": [c[1] for c in per_rank_cross],
                "note": ("device-side time per fit() iteration that the rank's first slice spun on "
                         "the left rank's hand-off granules (halo) and its last slice on the right "
                         "rank's back channel (status words 11 / 12, s_memrealtime); 0 on one GPU")},
            "scaling_model": scaling_model(n, T_total, world, int(getattr(eng, "spec_depth", 1)),
                                           pipelined),
            "build": _lib_provenance(),
            "iteration_roofline_frac": b_iter / (dt / args.steps) / (world * HBM_PEAK_GBS * 1e9),
            "cpu_baseline": cpu,
            "secondary": secondary,
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
