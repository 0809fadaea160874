"""GPU parity: the HIP path (libame_amd.so) against the reference's own outputs
(golden fixtures captured by tests/golden/make_golden.py) and against the CPU
oracle (oracle/ame_oracle.py).

Tolerances (stated here):
  * vs fp64 reference / fp64 oracle: ELBO and MSE relative 2e-6, means
    absolute 2e-6 * max(1, max|mu|), covariances absolute 1e-6 * max(1, max|S|).
    The device keeps means/covariances in fp32 storage and solves in fp64, so
    this is fp32 storage rounding amplified over a few iterations.
  * vs fp32 reference: 10x looser (the fp32 reference itself differs from the
    fp64 reference by up to 1.6e-5 on the means at n=40, lr=1).
"""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden, golden_params

pytestmark = pytest.mark.gpu

CFG = {"c1": (15, 10, 2), "tfix": (10, 5, 2), "mid": (40, 12, 3)}


def _make(tag):
    from ame_amd import TemporalAMEModel
    n, T, r = CFG[tag]
    m = TemporalAMEModel(n, T, r, ar_coefficient=0.8, rho_dyadic=0.5, seed=42)
    m.generate_data()
    return m


def _vi(model, method, lr, dev, **opts):
    from ame_amd import TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    if method == "naive":
        return TemporalAMENaiveMFVI(model, learning_rate=lr, device=dev, engine_options=opts)
    return TemporalAMEStructuredMFVI(model, factorization=method, learning_rate=lr, device=dev,
                                     engine_options=opts)


def _fixtures():
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "*_lr*.npz"))):
        name = os.path.basename(f)
        if name.endswith("_f64.npz"):
            continue
        tag, method = name.split("_")[:2]
        lr = float(name.split("_lr")[1].replace(".npz", ""))
        out.append((tag, method, lr, name))
    return out


@pytest.mark.parametrize("tag,method,lr,name", _fixtures())
def test_golden_trajectory(tag, method, lr, name, gpu_device):
    z32 = golden(name)
    f64 = name.replace(".npz", "_f64.npz")
    z = golden(f64) if os.path.exists(os.path.join(GOLDEN, f64)) else z32
    k = 1.0 if z is not z32 else 10.0
    m = _make(tag)
    vi = _vi(m, method, lr, gpu_device)
    assert np.array_equal(vi.X_mean.numpy(), z32["init_mean"])
    assert np.array_equal(vi.X_cov.numpy(), z32["init_cov"])
    iters = int(z["iters"])
    for it in range(1, iters + 1):
        vi.fit(max_iter=1, tolerance=0.0, verbose=False)
        if f"mean_{it}" in z:
            ref = z[f"mean_{it}"]
            err = np.abs(vi.X_mean.numpy().astype(np.float64) - ref).max()
            assert err <= k * 2e-6 * max(1.0, np.abs(ref).max()), (it, err)
        if f"cov_{it}" in z:
            ref = z[f"cov_{it}"]
            err = np.abs(vi.X_cov.numpy().astype(np.float64) - ref).max()
            assert err <= k * 1e-6 * max(1.0, np.abs(ref).max()), (it, err)
    e = np.array([float(x) for x in vi.history["elbo"]])
    rec = np.array(vi.history["reconstruction_error"])
    assert np.all(np.abs(e - z["elbo"]) <= k * 2e-6 * np.abs(z["elbo"])), (e, z["elbo"])
    assert np.all(np.abs(rec - z["recon"]) <= k * 2e-6 * np.abs(z["recon"])), (rec, z["recon"])
    sp = vi.elbo_terms()
    got = np.array([sp["loglik"], sp["prior0"], sp["trans"], sp["entropy"]])
    ref = z["elbo_split"][-1]
    assert np.all(np.abs(got - ref) <= k * 2e-6 * np.abs(z["elbo"][-1])), (got, ref)


def test_demo_100_iterations(gpu_device):
    """demo.py settings (lr=0.01, 100 iterations) for all three methods."""
    z = golden("c1_demo100.npz")
    for method in ("good", "bad", "naive"):
        m = _make("c1")
        vi = _vi(m, method, 0.01, gpu_device)
        h = vi.fit(max_iter=100, verbose=False)
        e = np.array([float(x) for x in h["elbo"]])
        ref = z[f"{method}_elbo"]
        assert len(e) == len(ref)
        assert np.all(np.abs(e - ref) <= 2e-5 * np.abs(ref)), method
        assert np.allclose(h["reconstruction_error"], z[f"{method}_recon"], rtol=2e-5, atol=0)
        assert np.abs(vi.X_mean.numpy() - z[f"{method}_mean"]).max() < 2e-4


def test_single_node_update(gpu_device):
    """Observation terms / one node update at init (structured_mf.py:289-326)."""
    z = golden("c1_single_step.npz")
    import ame_oracle as O
    P = golden_params("c1")
    m = _make("c1")
    Y = m.Y.numpy().astype(np.float64)
    for method in ("good", "bad"):
        Xm = z[f"{method}_before_mean"].astype(np.float64)
        for (i, t), Pr, hr in zip(z[f"{method}_obs_it"], z[f"{method}_obs_P"], z[f"{method}_obs_h"]):
            Po, ho = O.observation_terms(Y, Xm, P["R_inv"], int(i), int(t))
            assert np.allclose(Po, Pr, rtol=1e-5, atol=1e-4)
            assert np.allclose(ho, hr, rtol=1e-5, atol=1e-4)
    # one full sweep on the GPU: node 0 must equal the reference's _update_node_i(0)
    for method in ("good", "bad"):
        vi = _vi(_make("c1"), method, 1.0, gpu_device)
        vi.fit(max_iter=1, tolerance=0.0, verbose=False)
        ref = z[f"{method}_after0_mean"][0]
        assert np.abs(vi.X_mean.numpy()[0] - ref).max() < 2e-5


@pytest.mark.parametrize("n,T,r,method,lr", [
    (33, 7, 1, "good", 0.5), (64, 16, 4, "good", 0.01), (50, 9, 5, "bad", 1.0),
    (48, 6, 8, "naive", 0.3), (70, 5, 6, "good", 1.0), (40, 4, 16, "good", 0.01),
    (20, 1, 2, "good", 1.0), (2, 3, 2, "bad", 0.7), (24, 3, 7, "naive", 1.0),
    (1000, 2, 16, "good", 0.5), (700, 3, 8, "naive", 1.0), (900, 2, 16, "bad", 0.2),
    (60, 3, 12, "good", 0.5), (50, 3, 24, "bad", 0.7), (30, 2, 24, "naive", 1.0),
    (1200, 1, 24, "good", 0.3),
    # latent dims outside round 1's compiled set (each split-build part)
    (40, 3, 10, "good", 0.5), (30, 2, 13, "naive", 1.0), (26, 3, 20, "bad", 0.7),
    (20, 2, 31, "good", 0.3), (33, 2, 9, "good", 1.0), (18, 2, 27, "naive", 0.5),
    (300, 2, 11, "good", 0.5)])
def test_vs_oracle_fp64(n, T, r, method, lr, gpu_device):
    """Random configurations (odd r, T=1, n=2, ...) against the fp64 oracle.

    Bound: 5e-6 relative, or -- where the problem itself amplifies fp32
    round-off (lr=1, larger r) -- no further from the fp64 oracle than the
    reference's own fp32 arithmetic (the fp32 oracle) is."""
    import ame_oracle as O
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(n, T, r, seed=7)
    m.generate_data_fast(seed=11)
    vi = _vi(m, method, lr, gpu_device)
    Xm = vi.X_mean.numpy().astype(np.float64).copy()
    Xc = vi.X_cov.numpy().astype(np.float64).copy()
    params = {k: getattr(m, k).numpy().astype(np.float64)
              for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")}
    Y = m.Y.numpy().astype(np.float64)
    Xm32 = vi.X_mean.numpy().copy()
    Xc32 = vi.X_cov.numpy().copy()
    ref = O.fit(Y, Xm, Xc, params, method, lr, max_iter=2, tolerance=0.0)
    p32 = {k: v.astype(np.float32) for k, v in params.items()}
    O.fit(m.Y.numpy(), Xm32, Xc32, p32, method, lr, max_iter=2, tolerance=0.0)
    fp32_err = np.abs(Xm32.astype(np.float64) - Xm).max()
    h = vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    err = np.abs(vi.X_mean.numpy() - Xm).max()
    assert err <= max(5e-6 * max(1.0, np.abs(Xm).max()), fp32_err), (err, fp32_err)
    cerr = np.abs(vi.X_cov.numpy() - Xc).max()
    assert cerr <= 1e-6 * max(1.0, np.abs(Xc).max()), cerr
    for a, b in zip(h["elbo"], ref["elbo"]):
        assert abs(float(a) - b) <= 5e-6 * abs(b), (float(a), b)
    for a, b in zip(h["reconstruction_error"], ref["reconstruction_error"]):
        assert abs(a - b) <= 5e-6 * abs(b), (a, b)


def test_not_swap_consistent(gpu_device):
    """Y mutated after generation (multiplicative_strength_comparison.py:161-186
    does this): the ELBO/MSE must read both triangles."""
    import ame_oracle as O
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(30, 4, 3, seed=3)
    m.generate_data_fast(seed=5)
    m.Y[3, 7, 1, 0] += 0.5
    m.Y[20, 2, 3, 1] -= 0.25
    vi = _vi(m, "good", 0.2, gpu_device)
    assert not vi.engine.swap_consistent
    Xm = vi.X_mean.numpy().astype(np.float64).copy()
    Xc = vi.X_cov.numpy().astype(np.float64).copy()
    params = {k: getattr(m, k).numpy().astype(np.float64)
              for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")}
    ref = O.fit(m.Y.numpy().astype(np.float64), Xm, Xc, params, "good", 0.2, 1, 0.0)
    h = vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    assert abs(h["reconstruction_error"][0] - ref["reconstruction_error"][0]) <= 5e-6 * ref["reconstruction_error"][0]
    assert abs(float(h["elbo"][0]) - ref["elbo"][0]) <= 5e-6 * abs(ref["elbo"][0])


def test_deterministic(gpu_device):
    from ame_amd import TemporalAMEModel
    outs = []
    for _ in range(2):
        m = TemporalAMEModel(96, 12, 4, seed=1)
        m.generate_data_fast(seed=2)
        vi = _vi(m, "good", 0.5, gpu_device)
        h = vi.fit(max_iter=2, tolerance=0.0, verbose=False)
        outs.append((vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy(),
                     [float(e) for e in h["elbo"]], list(h["reconstruction_error"])))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2] and outs[0][3] == outs[1][3]


def _twins(n, T, r, method, lr, dev, **opts):
    """Two identical runs: the engine's speculative schedule (with `opts`) and
    the in-order one."""
    from ame_amd import TemporalAMEModel
    out = []
    for spec in (True, False):
        m = TemporalAMEModel(n, T, r, seed=3)
        m.generate_data_fast(seed=4)
        vi = _vi(m, method, lr, dev, **(opts if spec else {"speculate": False}))
        out.append(vi)
    return out


def test_speculative_sweep_is_exact(gpu_device):
    """The next sweep started beside the ELBO kernels: bit-identical states and
    histories to running every kernel in order."""
    a, b = _twins(80, 9, 4, "good", 0.3, gpu_device)
    ha = a.fit(max_iter=5, tolerance=0.0, verbose=False)
    hb = b.fit(max_iter=5, tolerance=0.0, verbose=False)
    assert np.array_equal(a.X_mean.numpy(), b.X_mean.numpy())
    assert np.array_equal(a.X_cov.numpy(), b.X_cov.numpy())
    assert [float(e) for e in ha["elbo"]] == [float(e) for e in hb["elbo"]]
    assert ha["reconstruction_error"] == hb["reconstruction_error"]


def test_speculation_dropped_on_convergence(gpu_device):
    """fit() stops at convergence: the started sweep leaves no trace, and a later
    fit() continues exactly like the in-order run."""
    a, b = _twins(60, 7, 3, "naive", 0.5, gpu_device)
    for vi in (a, b):
        vi.fit(max_iter=10, tolerance=1.0, verbose=False)   # converges at iteration 3
    assert len(a.history["elbo"]) == len(b.history["elbo"]) == 4
    assert np.array_equal(a.X_mean.numpy(), b.X_mean.numpy())
    assert np.array_equal(a.X_cov.numpy(), b.X_cov.numpy())
    for vi in (a, b):
        vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    assert np.array_equal(a.X_mean.numpy(), b.X_mean.numpy())
    assert np.array_equal(a.X_cov.numpy(), b.X_cov.numpy())
    assert [float(e) for e in a.history["elbo"]] == [float(e) for e in b.history["elbo"]]


def test_pipelined_sweeps_many_slices(gpu_device):
    """100 slices: consecutive sweeps overlap slice by slice (done flags); the
    result is bit-identical to the in-order schedule."""
    a, b = _twins(150, 100, 4, "good", 0.5, gpu_device)
    assert a.engine.pipelined
    ha = a.fit(max_iter=4, tolerance=0.0, verbose=False)
    hb = b.fit(max_iter=4, tolerance=0.0, verbose=False)
    assert np.array_equal(a.X_mean.numpy(), b.X_mean.numpy())
    assert np.array_equal(a.X_cov.numpy(), b.X_cov.numpy())
    assert [float(e) for e in ha["elbo"]] == [float(e) for e in hb["elbo"]]


@pytest.mark.parametrize("depth", [1, 3, 5])
def test_speculation_depth_is_exact(depth, gpu_device):
    """Sweeps queued `depth` deep (state ring of depth + 1 slots, each slice
    waiting on the device for the previous sweep): bit-identical to the
    in-order schedule, also when fit() stops at convergence with sweeps still
    queued, and when a later fit() continues."""
    a, b = _twins(90, 40, 4, "good", 0.5, gpu_device, spec_depth=depth)
    assert a.engine.spec_depth == depth and len(a.engine.xs) == depth + 1
    ha = a.fit(max_iter=7, tolerance=0.0, verbose=False)
    hb = b.fit(max_iter=7, tolerance=0.0, verbose=False)
    assert [float(e) for e in ha["elbo"]] == [float(e) for e in hb["elbo"]]
    for vi in (a, b):
        vi.fit(max_iter=10, tolerance=1.0, verbose=False)   # stops at its 4th iteration
        vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    assert np.array_equal(a.X_mean.numpy(), b.X_mean.numpy())
    assert np.array_equal(a.X_cov.numpy(), b.X_cov.numpy())
    assert [float(e) for e in a.history["elbo"]] == [float(e) for e in b.history["elbo"]]


def test_unpipelined_queue_is_one_deep(gpu_device):
    """Sweeps that do not order themselves on the device (pipeline=False) are
    queued one deep whatever spec_depth asks, and stay exact."""
    a, b = _twins(90, 40, 4, "good", 0.5, gpu_device, pipeline=False, spec_depth=2)
    assert not a.engine.pipelined and a.engine.spec_depth == 1
    ha = a.fit(max_iter=5, tolerance=0.0, verbose=False)
    hb = b.fit(max_iter=5, tolerance=0.0, verbose=False)
    assert np.array_equal(a.X_mean.numpy(), b.X_mean.numpy())
    assert np.array_equal(a.X_cov.numpy(), b.X_cov.numpy())
    assert [float(e) for e in ha["elbo"]] == [float(e) for e in hb["elbo"]]


def test_pipelined_sweep_after_device_state_write(gpu_device):
    """A pipelined sweep started right after the state was written on the main
    stream (set_means from a device tensor, queued behind a long kernel) reads
    the written state: its only device-side wait is on the previous sweep, so
    the launch also waits for the host-issued writes (_mark_host_writes)."""
    a, b = _twins(150, 20, 4, "good", 0.5, gpu_device)
    assert a.engine.pipelined
    for vi in (a, b):
        vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    X = a.X_mean.clone()
    X[:, :, 0] += 0.25
    outs = []
    for vi in (a, b):
        eng = vi.engine
        big = torch.randn(4096, 4096, device=gpu_device)
        for _ in range(8):   # keep the main stream busy well past the launch
            big = big @ big.T * 1e-3
        eng.set_means(X.to(gpu_device))
        eng.terms(speculate=1 if eng.speculation else 0)
        eng.sweep()
        eng.terms()
        outs.append((eng.means_local().cpu().clone(), eng.covs_local().cpu().clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_engine_dropped_with_sweep_queued(gpu_device):
    """An engine dropped while a started sweep still runs: the sweep streams are
    recorded on every buffer a launch passes as a raw pointer, so the caching
    allocator does not hand that memory to the next engine early; the next fit of
    the same shape is bit-identical to the in-order schedule."""
    import gc
    a, _ = _twins(150, 20, 4, "good", 0.5, gpu_device)
    a.fit(max_iter=1, tolerance=0.0, verbose=False)
    a.engine.speculate(1)
    del a, _
    gc.collect()
    b, c = _twins(150, 20, 4, "good", 0.5, gpu_device)
    b.fit(max_iter=2, tolerance=0.0, verbose=False)
    c.fit(max_iter=2, tolerance=0.0, verbose=False)
    assert np.array_equal(b.X_mean.numpy(), c.X_mean.numpy())
    assert np.array_equal(b.X_cov.numpy(), c.X_cov.numpy())


def test_state_attributes_stay_live(gpu_device):
    """X = vi.X_mean taken before fit() sees the fitted values once the
    attribute is read again (reference getters return the live tensor,
    structured_mf.py:328-338); a later host edit still goes to the device."""
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(40, 6, 3, seed=9)
    m.generate_data_fast(seed=9)
    vi = _vi(m, "good", 0.5, gpu_device)
    X, S = vi.X_mean, vi.X_cov
    x0 = X.clone()
    vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    assert vi.X_mean is X and vi.X_cov is S
    assert not torch.equal(X, x0)
    assert torch.equal(vi.get_variational_means(), X)
    X[0, 0, 0] += 1.0                      # host edit -> uploaded before the next step
    vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    assert vi.engine.x_a.shape[1] == 40


@pytest.mark.parametrize("group", [3, 4])
def test_slice_groups_are_exact(group, gpu_device):
    """Local slices launched as consecutive groups (slice_group forces the
    size; by default only when T_local exceeds the co-resident workgroups):
    bit-identical to one launch over all slices."""
    from ame_amd import TemporalAMEModel
    outs = []
    for g in (0, group):
        m = TemporalAMEModel(48, 10, 3, seed=12)
        m.generate_data_fast(seed=12)
        vi = _vi(m, "good", 0.5, gpu_device, slice_group=g)
        assert len(vi.engine.groups) == (1 if g == 0 else -(-10 // g))
        # groups of a pipelined kernel alternate streams and overlap on the device
        assert vi.engine.pipelined
        h = vi.fit(max_iter=3, tolerance=0.0, verbose=False)
        outs.append((vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy(), [float(e) for e in h["elbo"]]))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]
