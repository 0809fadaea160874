"""BASELINE config 5's own workload on ONE MI355X: n=4096, T=256, r=32 (d=66),
Naive-MF vs SMF-good vs SMF-bad on the same Y (experiments/three_way_conparison.py:141-179).

The 256 slices exceed the co-resident workgroups of the GEMV-worker sweep
(kind 22: 8 workgroups per slice, 32 slices fill the chip), so every sweep
runs as 8 consecutive slice groups of 32 (engine.slice_groups); group g+1's
first slice takes group g's last slice's new means from its hand-off
granules, so the 255 slice boundaries carry the Gauss-Seidel order exactly as
one launch would (reference: the t loop of structured_mf.py:240 has no limit
on T).  The same test on the pipelined kind 23 (11 overlapping groups of
23-24, 1 100 nodes against the oracle) is profiles/r05_i_pytest_pipe_and_c5full_kind23.txt.
Per variant, two fit() iterations; checks:

* kind 22, 8 groups, in order (not pipelined);
* the second sweep against the fp64 oracle's replay from the device's state
  after the first (ame_oracle.sweep_stats, pinned in tests/test_oracle_fast.py):
  nodes 0..K-1 of ALL 256 slices -- 600 nodes for SMF-good (past the first
  GEMV worker's 585-node range, so the hand-over to the second worker is
  checked), 64 for bad / naive (past the workers' 4-node look-behind); means within 5e-6 * max(1, |mu|), covariances 1e-6 * max(1, |S|);
* the device ELBO / MSE of the final state against an fp64 evaluation of that
  state slice by slice (tests/elbo_check.py: torch's own fp64 kernels on the
  GPU for all 256 slices -- the CPU would need ~10 minutes for the 3 x 256
  n x n residual matrices -- and that evaluation pinned to the same code on
  the CPU on slices 0, 1, 128, 255 of every variant), 5e-6 relative.

Reference: naive_mf.py:207-282, structured_mf.py:211-326, :115-209,
temporal_ame.py:255-291.
"""
import gc
import time

import numpy as np
import pytest
import torch

from test_gpu_baseline_shapes import _params, _vi

pytestmark = pytest.mark.gpu

N, T, R, LR = 4096, 256, 32, 0.01
KF = {"good": 600, "bad": 64, "naive": 64}
PIN_SLICES = (0, 1, 128, 255)


def _rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


@pytest.mark.timeout(900)
def test_config5_full_workload_three_way(gpu_device):
    import ame_oracle as O
    from elbo_check import assemble, cov_sums, pair_sums
    from ame_amd import TemporalAMEModel, _lib
    t_start = time.time()
    m = TemporalAMEModel(N, T, R, seed=42)
    m.generate_data_fast(device=gpu_device, seed=42)
    p64 = _params(m)
    YK = m.Y[:max(KF.values())].cpu().numpy()     # rows the oracle replay reads
    print(f"config 5 full: data ready ({time.time() - t_start:.0f} s)", flush=True)
    finals, dev_terms, cov_s = {}, {}, {}
    for method in ("naive", "good", "bad"):
        t0 = time.time()
        vi = _vi(m, method, LR, gpu_device)
        eng = vi.engine
        # the GEMV-worker sweep in 8 consecutive groups of 32 slices
        assert eng.sweep_kind == _lib.AME_SWEEP_V2_WORKERS
        assert len(eng.groups) == 8 and {s for _, s in eng.groups} == {32}, eng.groups
        assert not eng.pipelined
        kf = KF[method]
        vi.fit(max_iter=1, tolerance=0.0, verbose=False)
        x1 = eng.means_local().cpu().numpy().astype(np.float64)
        c1 = eng.covs_local()[:kf].cpu().numpy().astype(np.float64)
        h = vi.fit(max_iter=1, tolerance=0.0, verbose=False)
        got_m = eng.means_local().cpu().numpy()
        got_c = eng.covs_local()[:kf].cpu().numpy()
        # covariance sums of the final state, slice by slice on the device (fp64
        # torch), and on the CPU for the pin slices
        cov_s[method] = cov_sums(lambda t: eng.cov[t], T, p64, device=gpu_device)
        pin_gpu = cov_sums(lambda t: eng.cov[t], T, p64, device=gpu_device, ts=PIN_SLICES)
        pin_cpu = cov_sums(lambda t: eng.cov[t], T, p64, device="cpu", ts=PIN_SLICES)
        for k in pin_cpu:
            assert _rel(pin_gpu[k], pin_cpu[k]) <= 1e-10, (k, pin_gpu[k], pin_cpu[k])
        finals[method] = got_m
        dev_terms[method] = (float(h["elbo"][-1]), float(h["reconstruction_error"][-1]))
        del vi, eng
        gc.collect()
        torch.cuda.empty_cache()
        # the second sweep, nodes 0..kf-1 of all 256 slices, against the oracle
        O.sweep_stats(YK, x1, c1, p64, method, LR, nodes=range(kf))
        err = np.abs(got_m[:kf].astype(np.float64) - x1[:kf]).max()
        cerr = np.abs(got_c.astype(np.float64) - c1).max()
        print(f"config 5 full {method}: nodes 0..{kf - 1} x {T} slices vs fp64 oracle: "
              f"max|dmean| {err:.3e} (max|mean| {np.abs(x1[:kf]).max():.3f}), "
              f"max|dcov| {cerr:.3e} ({time.time() - t0:.0f} s)", flush=True)
        assert err <= 5e-6 * max(1.0, np.abs(x1[:kf]).max()), err
        assert cerr <= 1e-6 * max(1.0, np.abs(c1).max()), cerr
        del x1, c1, got_c
    # the Y side of all three ELBOs in one pass over the slices
    order = ("naive", "good", "bad")
    states = [finals[k] for k in order]
    pairs = pair_sums(lambda t: m.Y[:, :, t], states, p64, device=gpu_device)
    pin_gpu = pair_sums(lambda t: m.Y[:, :, t], states, p64, device=gpu_device, ts=PIN_SLICES)
    pin_cpu = pair_sums(lambda t: m.Y[:, :, t], states, p64, device="cpu", ts=PIN_SLICES)
    for g, c in zip(pin_gpu, pin_cpu):
        assert _rel(g[0], c[0]) <= 1e-10 and _rel(g[1], c[1]) <= 1e-10, (g, c)
    for k, (quad, sq) in zip(order, pairs):
        e = assemble(finals[k], cov_s[k], quad, sq, p64, k)
        elbo, mse = dev_terms[k]
        print(f"config 5 full {k}: device ELBO {elbo:.8e} vs fp64 {e['elbo']:.8e}, "
              f"MSE {mse:.8e} vs {e['recon']:.8e}", flush=True)
        assert _rel(elbo, e["elbo"]) <= 5e-6, (k, elbo, e)
        assert _rel(mse, e["recon"]) <= 5e-6, (k, mse, e)
    print(f"config 5 full: {time.time() - t_start:.0f} s", flush=True)
