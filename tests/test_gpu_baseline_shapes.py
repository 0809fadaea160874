"""GPU parity at the BASELINE.json configuration shapes, through the C-ABI.

* config 2 (n=256, T=64, r=8): the whole fit (2 iterations, good / bad /
  naive) against the fp64 oracle;
* config 3 (n=1024, T=128, r=16, lr=0.01 -- the bench workload): the
  production schedule (speculative, pipelined sweeps queued two deep) is bit
  for bit the in-order schedule, and the in-order run's third sweep -- ALL
  1024 nodes x 128 slices, means and covariances -- against the fp64 oracle
  replaying that sweep from the device's state after two iterations
  (ame_oracle.sweep_stats, pinned to the direct restatement and the
  reference's fp64 runs in tests/test_oracle_fast.py), plus its first K nodes
  against the direct fp64 / fp32 restatement; the device ELBO / MSE of the
  full state against the oracle's ELBO of the same state;
* config 4's per-rank shape (n=1024, T_local=64, r=16): two time-sharded
  ranks on one GPU reproduce the single-process T=128 run bit for bit;
* config 4 at full T (n=1024, T=512, r=16) in one process: the third sweep,
  all 1024 x 512, against the fp64 oracle's replay.

Reference: structured_mf.py:211-326 (sweep), :115-209 (ELBO),
naive_mf.py:207-282, temporal_ame.py:255-291 (MSE).

Tolerances as in test_gpu_parity.py: means within 5e-6 * max(1, |mu|) of the
fp64 oracle or no further from it than the reference's own fp32 arithmetic
(the fp32 oracle) is; covariances 1e-6 * max(1, |S|); ELBO / MSE 5e-6 relative.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

PKEYS = ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")


def _vi(model, method, lr, dev, distributed=None, **opts):
    from ame_amd import TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    if method == "naive":
        return TemporalAMENaiveMFVI(model, learning_rate=lr, device=dev, distributed=distributed,
                                    engine_options=opts)
    return TemporalAMEStructuredMFVI(model, factorization=method, learning_rate=lr, device=dev,
                                     distributed=distributed, engine_options=opts)


def _params(m, dtype=np.float64):
    return {k: getattr(m, k).cpu().numpy().astype(dtype) for k in PKEYS}


@pytest.mark.parametrize("method", ["good", "bad", "naive"])
def test_config2_full_fit(method, gpu_device):
    """BASELINE config 2 at full size: 2 fit iterations vs the fp64 oracle."""
    import ame_oracle as O
    from ame_amd import TemporalAMEModel
    n, T, r, lr = 256, 64, 8, 0.01
    m = TemporalAMEModel(n, T, r, seed=42)
    m.generate_data_fast(seed=42)
    vi = _vi(m, method, lr, gpu_device)
    Xm = vi.X_mean.numpy().astype(np.float64).copy()
    Xc = vi.X_cov.numpy().astype(np.float64).copy()
    Xm32, Xc32 = vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()
    ref = O.fit(m.Y.numpy().astype(np.float64), Xm, Xc, _params(m), method, lr, 2, 0.0)
    O.fit(m.Y.numpy(), Xm32, Xc32, _params(m, np.float32), method, lr, 2, 0.0)
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


def _config3(dev):
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(1024, 128, 16, seed=42)
    m.generate_data_fast(device=dev, seed=42)
    return m


def test_config3_schedule_prefix_and_elbo(gpu_device):
    """BASELINE config 3 (the bench workload) at its own shape."""
    import ame_oracle as O
    n, T, r, lr, K = 1024, 128, 16, 0.01, 8
    # production schedule: one fit() call, sweeps started ahead and pipelined
    m = _config3(gpu_device)
    prod = _vi(m, "good", lr, gpu_device)
    assert prod.engine.pipelined and prod.engine.spec_depth == 2   # derived: 1 GPU, T = 128
    hp = prod.fit(max_iter=3, tolerance=0.0, verbose=False)
    prod_mean = prod.X_mean.numpy().copy()
    prod_cov_digest = hashlib.sha256(prod.X_cov.numpy().tobytes()).hexdigest()
    del prod
    torch.cuda.empty_cache()
    # in-order schedule, one iteration per fit() call, no speculation
    m = _config3(gpu_device)
    vi = _vi(m, "good", lr, gpu_device, speculate=False)
    vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    Xm = vi.X_mean.numpy().astype(np.float64).copy()
    Xc = vi.X_cov.numpy().astype(np.float64).copy()
    Xm32, Xc32 = vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()
    h = vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    got_m, got_c = vi.X_mean.numpy(), vi.X_cov.numpy()
    # the pipelined schedule is the in-order one, bit for bit
    assert np.array_equal(prod_mean, got_m)
    assert prod_cov_digest == hashlib.sha256(got_c.tobytes()).hexdigest()
    assert [float(e) for e in hp["elbo"]] == [float(e) for e in h["elbo"]]
    assert hp["reconstruction_error"] == h["reconstruction_error"]
    # sweep 3, nodes 0..K-1 of every slice, against the oracle's replay
    Ycpu = m.Y.cpu().numpy()
    Y64 = Ycpu.astype(np.float64)
    p64, p32 = _params(m), _params(m, np.float32)
    c64, c32 = O.prior_terms(p64, T, np.float64), O.prior_terms(p32, T, np.float32)
    for i in range(K):
        O.update_node(Y64, Xm, Xc, p64, i, "good", lr, c64)
        O.update_node(Ycpu, Xm32, Xc32, p32, i, "good", lr, c32)
    fp32_err = np.abs(Xm32[:K].astype(np.float64) - Xm[:K]).max()
    err = np.abs(got_m[:K].astype(np.float64) - Xm[:K]).max()
    assert err <= max(5e-6 * max(1.0, np.abs(Xm[:K]).max()), fp32_err), (err, fp32_err)
    cerr = np.abs(got_c[:K].astype(np.float64) - Xc[:K]).max()
    assert cerr <= 1e-6 * max(1.0, np.abs(Xc[:K]).max()), cerr
    # the whole third sweep: every node of every slice (fp64 oracle)
    O.sweep_stats(Ycpu, Xm, Xc, p64, "good", lr, nodes=range(K, n))
    err_all = np.abs(got_m.astype(np.float64) - Xm).max()
    cerr_all = np.abs(got_c.astype(np.float64) - Xc).max()
    print(f"config 3 full sweep vs fp64 oracle: max|dmean| {err_all:.3e} "
          f"(max|mean| {np.abs(Xm).max():.3f}), max|dcov| {cerr_all:.3e}, "
          f"prefix fp32-arithmetic error {fp32_err:.3e}")
    assert err_all <= 5e-6 * max(1.0, np.abs(Xm).max()), err_all
    assert cerr_all <= 1e-6 * max(1.0, np.abs(Xc).max()), cerr_all
    # the ELBO / MSE kernels on the full device state
    e_ref = O.elbo(Y64, got_m, got_c, p64, "good")
    mse_ref = O.recon_error(Y64, got_m)
    assert abs(float(h["elbo"][-1]) - e_ref) <= 5e-6 * abs(e_ref), (float(h["elbo"][-1]), e_ref)
    assert abs(h["reconstruction_error"][-1] - mse_ref) <= 5e-6 * mse_ref


# ---------------- config 4 per-rank shape: 2 ranks x T_local=64 ----------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _c4_run(distributed):
    dev = torch.device("cuda", 0)
    m = _config3(dev)
    vi = _vi(m, "good", 0.01, dev, distributed=distributed)
    h = vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    mean = vi.X_mean.numpy().copy()
    digest = hashlib.sha256(vi.X_cov.numpy().tobytes()).hexdigest()
    return mean, digest, [float(e) for e in h["elbo"]], list(h["reconstruction_error"])


def _c4_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = _c4_run(True)
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def test_config4_rank_shape_two_ranks(gpu_device):
    """n=1024, r=16, T=128 split over 2 ranks (T_local=64, config 4's per-rank
    shape) on one GPU: bit-equal to the single-process run."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(rk, 2, port, q)) for rk in range(2)]
    for p in procs:
        p.start()
    try:
        result = q.get(timeout=110)
    except Exception:
        result = None
    for p in procs:
        p.join(timeout=30)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
            p.join()
    assert codes == [0, 0], f"rank exit codes {codes}"
    mean_d, dig_d, elbo_d, rec_d = result
    mean_s, dig_s, elbo_s, rec_s = _c4_run(False)
    assert np.array_equal(mean_d, mean_s)
    assert dig_d == dig_s
    assert np.allclose(elbo_d, elbo_s, rtol=1e-6, atol=0)
    assert np.allclose(rec_d, rec_s, rtol=1e-12, atol=0)


# ---------------- config 4 on one GPU: T=512 > co-resident slices ----------------
def _c4full_run(distributed, group):
    from ame_amd import TemporalAMEModel
    dev = torch.device("cuda", 0)
    m = TemporalAMEModel(1024, 512, 16, seed=42)
    m.generate_data_fast(device=dev, seed=42)
    vi = _vi(m, "good", 0.01, dev, distributed=distributed, slice_group=group)
    e = vi.engine
    groups = len(e.groups)
    # the co-residency rule: every spinning workgroup of every
    # rank on this GPU fits at once
    resid = (e.device_sharers, e.coresident_launches, max(sz for _, sz in e.groups), e.resident_slots)
    h = vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    mean = vi.X_mean.numpy().copy()
    digest = hashlib.sha256(vi.X_cov.numpy().tobytes()).hexdigest()
    return mean, digest, [float(e) for e in h["elbo"]], list(h["reconstruction_error"]), groups, resid


def _c4full_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the forced group of 128 is clamped to what 1/2 of the chip holds for
        # two pipelined launches (64): before round 6 it was not, and 2 ranks x 2
        # launches x 128 one-per-CU workgroups asked for 512 of 256 CUs
        # (profiles/r05_fin6_pytest_gpu_fail.txt)
        out = _c4full_run(True, 128)
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def test_config4_full_T_one_gpu(gpu_device):
    """BASELINE config 4 (n=1024, T=512, r=16) in one process on one GPU: the
    512 slices exceed the co-resident workgroups, so each sweep runs as
    consecutive slice groups; bit-equal to the same problem split over two
    time-sharded ranks."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4full_worker, args=(rk, 2, port, q)) for rk in range(2)]
    for p in procs:
        p.start()
    try:
        result = q.get(timeout=200)
    except Exception:
        result = None
    for p in procs:
        p.join(timeout=30)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
            p.join()
    assert codes == [0, 0], f"rank exit codes {codes}"
    mean_d, dig_d, elbo_d, rec_d, groups_d, resid_d = result
    mean_s, dig_s, elbo_s, rec_s, groups_s, resid_s = _c4full_run(False, 0)
    for sharers, launches, group, slots in (resid_d, resid_s):
        assert sharers * launches * group <= slots, (sharers, launches, group, slots)
    assert resid_d[0] == 2 and resid_s[0] == 1
    assert groups_s >= 2 and groups_d >= 2
    assert np.array_equal(mean_d, mean_s)
    assert dig_d == dig_s
    assert np.allclose(elbo_d, elbo_s, rtol=1e-6, atol=0)
    assert np.allclose(rec_d, rec_s, rtol=1e-12, atol=0)


# ---------------- config 5's per-rank shape (n=4096, T_local=32, r=32) ----------------
def _replay_prefix(Y32, x0, c0, params64, params32, method, lr, K, T):
    """The fp64 and fp32 oracle's replay of nodes 0..K-1 of one sweep from the
    pre-sweep state (node i depends only on that state and on nodes < i,
    SURVEY.md App. B).  Y stays fp32 (observation_terms promotes the row)."""
    import ame_oracle as O
    Xm, Xm32 = x0.astype(np.float64), x0.copy()
    Xc, Xc32 = c0[:K].astype(np.float64), c0[:K].copy()
    c64, c32 = O.prior_terms(params64, T, np.float64), O.prior_terms(params32, T, np.float32)
    for i in range(K):
        O.update_node(Y32, Xm, Xc, params64, i, method, lr, c64)
        O.update_node(Y32, Xm32, Xc32, params32, i, method, lr, c32)
    return Xm[:K], Xc, Xm32[:K].astype(np.float64)


def _check_prefix(got_m, got_c, ref_m, ref_c, ref_m32):
    fp32_err = np.abs(ref_m32 - ref_m).max()
    err = np.abs(got_m.astype(np.float64) - ref_m).max()
    assert err <= max(5e-6 * max(1.0, np.abs(ref_m).max()), fp32_err), (err, fp32_err)
    cerr = np.abs(got_c.astype(np.float64) - ref_c).max()
    assert cerr <= 1e-6 * max(1.0, np.abs(ref_c).max()), cerr
    return err, fp32_err


@pytest.mark.timeout(900)
@pytest.mark.parametrize("method", ["good", "bad", "naive"])
def test_config5_rank_shape(method, gpu_device):
    """BASELINE config 5 per rank: n=4096, T_local=32, r=32 (d=66), lr=0.01 --
    the v2 sweep with seven GEMV worker workgroups per slice on the full chip
    (32 x 8 = 256 workgroups).
    * the first K=12 nodes of every slice of the second sweep against the
      direct fp64 / fp32 restatement's replay (past the workers' look-behind:
      partial m uses node j's NEW mean for j <= m-4, so nodes 4..11 take that
      path);
    * the fp64 oracle's replay of that sweep (ame_oracle.sweep_stats): ALL
      4096 nodes of every slice for SMF-good, the first 600 for bad / naive --
      past the first GEMV worker's node range (n / 7 = 585 nodes, + the 4-node
      look-behind), so every worker's partials and the hand-over between two
      workers' ranges are checked against the oracle, not against another
      kernel; means within 5e-6 * max(1, |mu|), covariances 1e-6 * max(1, |S|);
    * the device ELBO / MSE of the final state against the CPU ELBO of that
      same state (tests/elbo_check.py, 5e-6 relative).
    Reference: naive_mf.py:207-282, structured_mf.py:211-326, :115-209."""
    import ame_oracle as O
    from elbo_check import elbo_and_mse
    from ame_amd import TemporalAMEModel, _lib
    n, T, r, lr, K = 4096, 32, 32, 0.01, 12
    m = TemporalAMEModel(n, T, r, seed=42)
    m.generate_data_fast(device=gpu_device, seed=42)
    vi = _vi(m, method, lr, gpu_device)
    assert vi.engine.sweep_kind == _lib.AME_SWEEP_V2_WORKERS and not vi.engine.pipelined
    vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    x1, c1 = vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()
    h = vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    got_m, got_c = vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()
    del vi
    torch.cuda.empty_cache()
    Y32 = m.Y.cpu().numpy()
    rm, rc, rm32 = _replay_prefix(Y32, x1, c1, _params(m), _params(m, np.float32), method, lr, K, T)
    _check_prefix(got_m[:K], got_c[:K], rm, rc, rm32)
    KF = n if method == "good" else 600
    Xm, Xc = x1.astype(np.float64), c1[:KF].astype(np.float64)
    for a in range(0, KF, 1024):   # chunks, with a progress line (about 25 s each)
        O.sweep_stats(Y32, Xm, Xc, _params(m), method, lr, nodes=range(a, min(KF, a + 1024)))
        print(f"config 5 {method}: oracle replay at node {min(KF, a + 1024)} of {KF}", flush=True)
    err = np.abs(got_m[:KF].astype(np.float64) - Xm[:KF]).max()
    cerr = np.abs(got_c[:KF].astype(np.float64) - Xc).max()
    print(f"config 5 {method}: nodes 0..{KF - 1} vs fp64 oracle: max|dmean| {err:.3e} "
          f"(max|mean| {np.abs(Xm[:KF]).max():.3f}), max|dcov| {cerr:.3e}")
    assert err <= 5e-6 * max(1.0, np.abs(Xm[:KF]).max()), err
    assert cerr <= 1e-6 * max(1.0, np.abs(Xc).max()), cerr
    del Xc
    e = elbo_and_mse(Y32, got_m, got_c, _params(m), method)
    assert abs(float(h["elbo"][-1]) - e["elbo"]) <= 5e-6 * abs(e["elbo"]), (float(h["elbo"][-1]), e)
    assert abs(h["reconstruction_error"][-1] - e["recon"]) <= 5e-6 * e["recon"]


# ---------------- config 4 at full T on one GPU: full oracle replay ----------------
@pytest.mark.timeout(600)
def test_config4_full_T_oracle(gpu_device):
    """BASELINE config 4 (n=1024, T=512, r=16, lr=0.01) in one process: the
    512 slices run as consecutive slice groups.  The third sweep -- ALL 1024
    nodes x 512 slices, means and covariances -- against the fp64 oracle's
    replay of that sweep from the device's state after two iterations
    (ame_oracle.sweep_stats, pinned in tests/test_oracle_fast.py), with config
    3's bounds; the first K=8 nodes also against the direct fp64 / fp32
    restatement; the device ELBO / MSE against the CPU ELBO of the device state.
    Reference: structured_mf.py:211-326, :115-209, temporal_ame.py:255-291."""
    import ame_oracle as O
    from elbo_check import elbo_and_mse
    from ame_amd import TemporalAMEModel
    n, T, r, lr, K = 1024, 512, 16, 0.01, 8
    m = TemporalAMEModel(n, T, r, seed=42)
    m.generate_data_fast(device=gpu_device, seed=42)
    vi = _vi(m, "good", lr, gpu_device)
    assert len(vi.engine.groups) >= 2
    vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    x2, c2 = vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy()
    h = vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    got_m, got_c = vi.X_mean.numpy(), vi.X_cov.numpy()
    Y32 = m.Y.cpu().numpy()
    rm, rc, rm32 = _replay_prefix(Y32, x2, c2, _params(m), _params(m, np.float32), "good", lr, K, T)
    _check_prefix(got_m[:K], got_c[:K], rm, rc, rm32)
    Xm, Xc = x2.astype(np.float64), c2.astype(np.float64)
    del x2, c2
    for a in range(0, n, 256):   # chunks, with a progress line
        O.sweep_stats(Y32, Xm, Xc, _params(m), "good", lr, nodes=range(a, min(n, a + 256)))
        print(f"config 4: oracle replay at node {min(n, a + 256)} of {n}", flush=True)
    err_all = np.abs(got_m.astype(np.float64) - Xm).max()
    cerr_all = np.abs(got_c.astype(np.float64) - Xc).max()
    print(f"config 4 full sweep (1024 x 512) vs fp64 oracle: max|dmean| {err_all:.3e} "
          f"(max|mean| {np.abs(Xm).max():.3f}), max|dcov| {cerr_all:.3e}")
    assert err_all <= 5e-6 * max(1.0, np.abs(Xm).max()), err_all
    assert cerr_all <= 1e-6 * max(1.0, np.abs(Xc).max()), cerr_all
    del Xm, Xc
    e = elbo_and_mse(Y32, got_m, got_c, _params(m), "good")
    assert abs(float(h["elbo"][-1]) - e["elbo"]) <= 5e-6 * abs(e["elbo"]), (float(h["elbo"][-1]), e)
    assert abs(h["reconstruction_error"][-1] - e["recon"]) <= 5e-6 * e["recon"]
