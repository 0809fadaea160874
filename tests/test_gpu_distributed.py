"""Time-sharded sweep on the GPU: 2-4 ranks (processes) on one MI355X, boundary
means handed over through peer buffers (fine-grained device memory exported
with an IPC handle, ame_peer_alloc / ame_peer_open) while the ranks' sweep
kernels run; with 3+ ranks a middle rank has both neighbours (left halo in,
right halo out and both back channels at once).  Pipelined sweeps are queued
spec_depth deep on every rank (derived from the global slice count by
DeviceEngine, DESIGN.md §5, or given explicitly).  Must reproduce the
single-process result bit for bit (means, covariances) and the ELBO/MSE to fp64
round-off.

Only the same-device IPC path runs here (one GPU per box): the ranks' peer
buffers live on one device.  The cross-device xGMI path (a neighbour's buffer on
another GPU) is the same code with the handle opened on another device; it has
not run on hardware in this repository's tests."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


V3, W22, P23 = 3, 22, 23   # _lib.AME_SWEEP_V3, _lib.AME_SWEEP_V2_WORKERS, _lib.AME_SWEEP_V2_PIPE


def _run(n, T, r, method, lr, iters, distributed, depth=None, kind=None):
    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    m = TemporalAMEModel(n, T, r, seed=21)
    m.generate_data_fast(seed=4)
    dev = torch.device("cuda", 0)
    opts = {} if depth is None else {"spec_depth": depth}
    if kind == P23:   # requested: AUTO picks kind 22 for these shapes
        opts["sweep_kernel"] = P23
    # distributed: True, or TimeShardHalo options plus "expect" (the peer kind
    # the links must end up with)
    dopt = distributed
    if isinstance(distributed, dict):
        dopt = {k: v for k, v in distributed.items() if k != "expect"}
    if method == "naive":
        vi = TemporalAMENaiveMFVI(m, learning_rate=lr, device=dev, distributed=dopt,
                                  engine_options=opts)
    else:
        vi = TemporalAMEStructuredMFVI(m, factorization=method, learning_rate=lr, device=dev,
                                       distributed=dopt, engine_options=opts)
    eng = vi.engine
    if kind is not None:
        assert eng.sweep_kind == kind, (eng.sweep_kind, kind)
    if distributed and depth is not None:
        assert eng.pipelined and eng.spec_depth == depth and len(eng.xs) == depth + 1
    h = vi.fit(max_iter=iters, tolerance=0.0, verbose=False)
    if distributed:   # every peer link passed the setup pre-flight (distributed.py)
        assert vi._halo.preflight_ok
        if isinstance(distributed, dict):
            want = distributed.get("expect", distributed.get("peer_mode"))
            assert vi._halo.peer_kind == want, (vi._halo.peer_kind, want, vi._halo.preflight_log)
    return (vi.X_mean.numpy().copy(), vi.X_cov.numpy().copy(),
            [float(e) for e in h["elbo"]], list(h["reconstruction_error"]))


def _worker(rank, world, port, args, q, dist_opt=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, T, r, method, lr, iters, depth, kind = args
        out = _run(n, T, r, method, lr, iters, dist_opt, depth, kind)
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,T,r,method,lr,iters,depth,kind", [
    (2, 64, 8, 4, "good", 0.5, 3, None, V3), (2, 40, 6, 3, "bad", 1.0, 3, None, V3),
    (2, 48, 5, 2, "naive", 0.3, 3, None, V3), (3, 50, 9, 3, "good", 0.5, 6, None, V3),
    (4, 40, 12, 4, "good", 0.7, 6, None, V3),
    # the queue depth the model gives at N = 8: 3 sweeps ahead
    # on 3 and 4 ranks, 8 iterations (several wraps of the state ring)
    (3, 60, 12, 4, "good", 0.5, 8, 3, V3), (4, 64, 16, 3, "bad", 0.8, 8, 3, V3),
    # config 5's sweep kernel (r = 32, d = 66: v2 + seven GEMV-worker workgroups
    # per slice) time-sharded: the left-halo poll of a rank's first slice beside
    # the workers' partial ring, 2 and 3 ranks, good / bad / naive, in-order
    # sweeps over several iterations (kind 22 does not pipeline)
    (2, 300, 8, 32, "good", 0.5, 3, None, W22), (3, 240, 12, 32, "bad", 0.7, 3, None, W22),
    (2, 200, 6, 32, "naive", 0.4, 4, None, W22), (3, 301, 9, 32, "good", 0.01, 3, None, W22),
    # the pipelined GEMV-worker sweep (kind 23) across ranks: pipelined sweeps,
    # back channels and halo granules between ranks, depth 2 and 3
    (2, 300, 8, 32, "good", 0.5, 5, None, P23), (3, 240, 12, 32, "bad", 0.7, 6, 3, P23),
    (2, 200, 6, 32, "naive", 0.4, 5, None, P23)])
def test_ranks_one_gpu(world, n, T, r, method, lr, iters, depth, kind):
    _ranks_vs_one_process(world, n, T, r, method, lr, iters, depth, kind, True)


@pytest.mark.parametrize("world,n,T,r,method,lr,iters,depth,kind", [
    (2, 64, 8, 4, "good", 0.5, 3, None, V3), (3, 60, 12, 4, "good", 0.5, 8, 3, V3),
    (2, 300, 8, 32, "good", 0.5, 3, None, W22), (2, 300, 8, 32, "bad", 0.5, 5, None, P23)])
def test_ranks_host_peer_buffers(world, n, T, r, method, lr, iters, depth, kind):
    """peer_mode "host" (distributed.py HostPeerBuffer, the fallback when the
    device-IPC links fail their pre-flight): halo granules and back channels in
    POSIX shared host memory registered on the device; bit-equal to one
    process like the IPC form."""
    _ranks_vs_one_process(world, n, T, r, method, lr, iters, depth, kind, {"peer_mode": "host"})


def _ranks_vs_one_process(world, n, T, r, method, lr, iters, depth, kind, dist_opt):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    args = (n, T, r, method, lr, iters, depth, kind)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, world, port, args, q, dist_opt)) for rk in range(world)]
    for p in procs:
        p.start()
    try:
        result = q.get(timeout=150)   # read before join: a large put blocks the child
    except Exception:
        result = None
    for p in procs:
        p.join(timeout=30)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
            p.join()
    assert codes == [0] * world, f"rank exit codes {codes}"
    mean_d, cov_d, elbo_d, rec_d = result
    n, T, r, method, lr, iters, _, kind = args
    mean_s, cov_s, elbo_s, rec_s = _run(n, T, r, method, lr, iters, False, kind=kind)
    dm = np.argwhere(mean_d != mean_s)
    assert len(dm) == 0, (f"{len(dm)} mean entries differ, max {np.abs(mean_d - mean_s).max():.3e}; "
                          f"(node, t) first {sorted({(int(a), int(b)) for a, b, _ in dm})[:12]}; "
                          f"slices {sorted({int(b) for _, b, _ in dm})}; "
                          f"ELBO 1-process {elbo_s} vs ranks {elbo_d}")
    assert np.array_equal(cov_d, cov_s)
    assert np.allclose(elbo_d, elbo_s, rtol=1e-6, atol=0)
    assert np.allclose(rec_d, rec_s, rtol=1e-12, atol=0)


def _preflight_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
        m = TemporalAMEModel(40, 6, 2, seed=3)
        m.generate_data_fast(seed=3)
        vi = TemporalAMEStructuredMFVI(m, learning_rate=0.5, device=torch.device("cuda", 0),
                                       distributed=True)
        vi.fit(max_iter=1, tolerance=0.0, verbose=False)
        halo = vi._halo
        assert halo.preflight_ok
        # a link that delivers the wrong word: rank 0 stores a sentinel addressed
        # to another owner into rank 1's halo; rank 1 must name the pair, rank 0
        # must learn of it from the all_reduce, and neither may hang
        if rank == 0:
            real = halo._sentinel
            halo._sentinel = lambda kind, writer, owner: real(kind, writer,
                                                              owner + 7 if kind == 1 else owner)
        msg = None
        try:
            halo._preflight(vi.engine, halo._peers)
        except RuntimeError as e:
            msg = str(e)
        # the buffers were zeroed after the check: the sweep still runs
        vi.fit(max_iter=1, tolerance=0.0, verbose=False)
        if rank == 0:
            halo._sentinel = real
        # a library error inside the pre-flight (ame_peer_probe fails on rank 1):
        # it must not raise before rank 1 reaches the barrier and the all_reduce,
        # so both ranks raise and neither waits for the process-group timeout
        from ame_amd import distributed as D
        real_lib = D._lib.lib

        class _FailProbe:
            def __init__(self, L):
                self._L = L

            def __getattr__(self, name):
                if name == "ame_peer_probe":
                    return lambda *a: -1
                return getattr(self._L, name)

        if rank == 1:
            D._lib.lib = lambda: _FailProbe(real_lib())
        msg2 = None
        try:
            halo._preflight(vi.engine, halo._peers)
        except RuntimeError as e:
            msg2 = str(e)
        D._lib.lib = real_lib
        q.put((rank, msg, msg2))
    finally:
        dist.destroy_process_group()


def test_preflight_detects_bad_link():
    """The setup pre-flight of the peer links (distributed.py _preflight) raises
    on both ranks, naming the failing pair on its owner, when the word that
    arrives is not the sentinel that was sent -- and when a library call of the
    pre-flight itself fails on one rank (both ranks still reach the collective,
    so neither hangs)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_preflight_worker, args=(rk, 2, port, q)) for rk in range(2)]
    for p in procs:
        p.start()
    got, got2 = {}, {}
    try:
        for _ in range(2):
            rank, msg, msg2 = q.get(timeout=150)
            got[rank] = msg
            got2[rank] = msg2
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
                p.join()
    assert [p.exitcode for p in procs] == [0, 0]
    assert got[1] is not None and "rank 0 -> rank 1 (left halo)" in got[1], got[1]
    assert got[0] is not None and "another rank" in got[0], got[0]
    # the failing probe: rank 1 names the call, rank 0 sees its back channel empty
    assert got2[1] is not None and "ame_peer_probe" in got2[1], got2[1]
    assert got2[0] is not None and "rank 1 -> rank 0 (back channel)" in got2[0], got2[0]


def _fallback_worker(rank, world, port, q):
    """peer_mode "auto" with the device-IPC buffers made to fail on rank 1: the
    ipc pre-flight raises on both ranks, both switch to host buffers."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ame_amd.distributed as D
        if rank == 1:
            class _NoIpc(D.PeerBuffer):
                def __init__(self, *a, **k):
                    raise RuntimeError("injected: device IPC unavailable")
            D.PeerBuffer = _NoIpc
        out = _run(64, 8, 4, "good", 0.5, 3, {"peer_mode": "auto", "expect": "host"})
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_ipc_failure_falls_back_to_host_buffers():
    """The auto peer mode: a rank whose device-IPC buffer cannot be made records
    it, the ipc pre-flight fails on EVERY rank (no rank sweeps over a half-made
    link), every rank switches to host buffers, and the fit is bit-equal to one
    process."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fallback_worker, args=(rk, 2, port, q)) for rk in range(2)]
    for p in procs:
        p.start()
    outs = {}
    try:
        for _ in range(2):
            rk, out = q.get(timeout=150)
            outs[rk] = out
    except Exception:
        pass
    for p in procs:
        p.join(timeout=30)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
            p.join()
    assert codes == [0, 0], f"rank exit codes {codes}"
    mean_s, cov_s, _, _ = _run(64, 8, 4, "good", 0.5, 3, False)
    assert np.array_equal(outs[0][0], mean_s) and np.array_equal(outs[0][1], cov_s)
