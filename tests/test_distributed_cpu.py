"""Time-sharded (multi-GPU) decomposition, exercised on CPU with gloo, world_size 2.

What the GPU path does per sweep (ame_amd/distributed.py) is replayed here with
the numpy oracle as the per-rank compute and gloo as the transport:
  * contiguous time blocks from ``shard_range``;
  * right halo: all_gather of every rank's first-slice OLD means before the sweep;
  * left halo: rank g-1 hands mu_{i, t_begin-1}^NEW to rank g node by node
    during the sweep (send/recv here; {epoch,value} granules on the GPU);
  * ELBO: per-rank 8 sums -> all_reduce -> ``engine.assemble``.
The sharded result must equal the unsharded oracle sweep bit for bit (same
operations in the same order) and the ELBO to 1e-12.  ``TimeShardHalo``'s
CPU-capable collectives (gather_time, allreduce_sums) are checked directly.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ame_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range():
    from ame_amd.distributed import shard_range
    for T in (2, 5, 128, 1024, 1001):
        for world in (1, 2, 3, 8):
            if T < world:
                with pytest.raises(ValueError):
                    shard_range(T, world, 0)
                continue
            blocks = [shard_range(T, world, r) for r in range(world)]
            assert blocks[0][0] == 0
            for (a, la), (b, _) in zip(blocks, blocks[1:]):
                assert a + la == b
            assert sum(l for _, l in blocks) == T
            assert max(l for _, l in blocks) - min(l for _, l in blocks) <= 1


def _setup(n, T, r, seed):
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    m = TemporalAMEModel(n, T, r, seed=seed)
    m.generate_data()
    vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=0.5)
    P = {k: getattr(m, k).numpy().astype(np.float64) for k in ("R", "R_inv", "Sigma", "Psi",
                                                               "Phi", "Q")}
    return (m.Y.numpy().astype(np.float64), vi.X_mean.numpy().astype(np.float64),
            vi.X_cov.numpy().astype(np.float64), P, m)


def _worker(rank, world, port, n, T, r, method, lr, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ame_amd.distributed import TimeShardHalo, shard_range
        from ame_amd.engine import Constants, assemble
        from test_model_api import _oracle_sums
        Y, Xm, Xc, P, m = _setup(n, T, r, seed=11)
        t0, TL = shard_range(T, world, rank)
        t1 = t0 + TL
        consts = O.prior_terms(P, T, np.float64)
        for _sweep in range(2):
            # right halo: old first-slice means of every rank
            first = torch.from_numpy(np.ascontiguousarray(Xm[:, t0]))
            firsts = [torch.empty_like(first) for _ in range(world)]
            dist.all_gather(firsts, first)
            if rank < world - 1:
                Xm[:, t1] = firsts[rank + 1].numpy()
            for i in range(n):
                if rank > 0:   # left halo: mu_{i, t0-1}^new from rank-1
                    buf = torch.empty(Xm.shape[2], dtype=torch.float64)
                    dist.recv(buf, src=rank - 1)
                    Xm[i, t0 - 1] = buf.numpy()
                for t in range(t0, t1):
                    O.update_step(Y, Xm, Xc, P, i, t, method, lr, consts, T_total=T)
                if rank < world - 1:
                    dist.send(torch.from_numpy(np.ascontiguousarray(Xm[i, t1 - 1])), dst=rank + 1)
        # ELBO over the local slices, prev = left halo final means
        prev = Xm[:, t0 - 1] if rank > 0 else None
        sums = _oracle_sums(O, Y[:, :, t0:t1], Xm[:, t0:t1], Xc[:, t0:t1], P, n, T, m.d,
                            t_lo=t0, prev=prev)
        halo = TimeShardHalo.create(T)
        assert (halo.shard.t_begin, halo.shard.T_local) == (t0, TL)
        tot = halo.allreduce_sums(torch.from_numpy(sums)).numpy()
        terms = assemble(tot, n, T, m.d, method, Constants(m))
        full_mean = halo.gather_time(torch.from_numpy(np.ascontiguousarray(Xm[:, t0:t1])), 1)
        full_cov = halo.gather_time(torch.from_numpy(np.ascontiguousarray(Xc[:, t0:t1])), 1)
        if rank == 0:
            q.put((full_mean.numpy(), full_cov.numpy(), terms))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,T,r,method,lr", [(9, 6, 2, "good", 0.5), (8, 5, 3, "bad", 1.0),
                                             (7, 4, 1, "naive", 0.3)])
def test_time_sharded_sweep_matches_unsharded(n, T, r, method, lr):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, world, port, n, T, r, method, lr, q))
             for rk in range(world)]
    for p in procs:
        p.start()
    try:
        result = q.get(timeout=240)   # read before join: a large put blocks the child
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
    mean_s, cov_s, terms = result
    Y, Xm, Xc, P, m = _setup(n, T, r, seed=11)
    for _ in range(2):
        O.sweep(Y, Xm, Xc, P, method, lr)
    assert np.array_equal(mean_s, Xm)
    assert np.array_equal(cov_s, Xc)
    ref = O.elbo_split(Y, Xm, Xc, P, method)
    got = [terms["loglik"], terms["prior0"], terms["trans"], terms["entropy"]]
    assert np.allclose(got, ref, rtol=1e-12, atol=1e-9)
    assert abs(terms["recon"] - O.recon_error(Y, Xm)) < 1e-12


def _sharers_worker(rank, world, port, same, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ame_amd.distributed import TimeShardHalo
        halo = TimeShardHalo.create(8 * world)
        # the device identity of each rank (host, PCI address, UUID) without a
        # GPU: every rank on one device, or ranks 0-1 / 2-3 on two devices
        halo.device_key = staticmethod(lambda dev: ("h", 0, 0 if same else rank // 2, 0, ""))

        class _Eng:
            dev = None
        q.put((rank, halo.device_sharers(_Eng()), halo.peer_mode))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("same", [True, False])
def test_device_sharers_counts_ranks_per_gpu(same):
    """TimeShardHalo.device_sharers (the engine's co-residency budget divisor,
    DESIGN.md §5): 4 gloo ranks, all on one device -> 4 each; two per device
    -> 2 each.  The default peer mode is "auto" (IPC, host fallback)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharers_worker, args=(rk, 4, port, same, q)) for rk in range(4)]
    for p in procs:
        p.start()
    got = dict((rk, (k, m)) for rk, k, m in (q.get(timeout=120) for _ in range(4)))
    for p in procs:
        p.join(timeout=30)
    assert [p.exitcode for p in procs] == [0] * 4
    assert all(m == "auto" for _, m in got.values())
    assert [got[r][0] for r in range(4)] == ([4] * 4 if same else [2] * 4)
