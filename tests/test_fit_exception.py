"""fit() that raises: the device VI must not enter a collective on the way out.

`fit()` calls `_fit_end(ok)` from its `finally:` (reference fit loop:
base.py:127-208).  On a normal return a time-sharded rank quiesces with a
barrier (no neighbour's dropped sweep may still store into its peer buffers);
when fit() raises, the other ranks may sit in a different collective (the
ELBO all_reduce), so the exception path only synchronises locally and lets
the original exception through.

CPU only: the engine and halo are stand-ins that record what is called; the
two-rank case runs real gloo collectives.
"""
import datetime
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _Eng:
    def __init__(self, log):
        self.log = log
        self.dev = "cpu"

    def discard_speculation(self):
        self.log.append("discard")


class _Halo:
    def __init__(self, log, barrier=False):
        self.log = log
        self.barrier = barrier

    def quiesce(self, eng):
        self.log.append("quiesce")
        if self.barrier:
            dist.barrier()

    def quiesce_local(self, eng):
        self.log.append("quiesce_local")


def _vi(log, fail_at=None, barrier=False, elbo_collective=False):
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI

    class VI(TemporalAMEStructuredMFVI):
        it = 0

        def _update_step(self):
            if fail_at is not None and self.it == fail_at:
                raise KeyError("injected")
            self.it += 1

        def _compute_elbo(self):
            if elbo_collective:
                t = torch.ones(1)
                dist.all_reduce(t)
            return torch.tensor(-1.0 * self.it)

        def _compute_reconstruction_error(self):
            return 0.0

    m = TemporalAMEModel(6, 3, 1, seed=1)
    m.generate_data()
    vi = VI(m, learning_rate=0.5)
    vi._engine = _Eng(log)
    vi._halo = _Halo(log, barrier)
    return vi


def test_fit_end_normal_return_quiesces():
    log = []
    vi = _vi(log)
    vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    assert log == ["discard", "quiesce"]


def test_fit_end_exception_is_local_and_propagates():
    log = []
    vi = _vi(log, fail_at=1)
    with pytest.raises(KeyError, match="injected"):
        vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    assert log == ["discard", "quiesce_local"]


def test_fit_end_exception_survives_failing_cleanup():
    """A faulted device makes the local synchronize raise too: the caller still
    sees fit()'s own exception."""
    log = []
    vi = _vi(log, fail_at=0)

    def boom(eng):
        raise RuntimeError("device fault")
    vi._halo.quiesce_local = boom
    with pytest.raises(KeyError, match="injected"):
        vi.fit(max_iter=2, tolerance=0.0, verbose=False)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2,
                            timeout=datetime.timedelta(seconds=20))
    log = []
    # rank 1 raises in its second sweep; rank 0 goes on into the ELBO all_reduce
    vi = _vi(log, fail_at=1 if rank == 1 else None, barrier=True, elbo_collective=True)
    err = None
    try:
        vi.fit(max_iter=4, tolerance=0.0, verbose=False)
    except Exception as e:  # noqa: BLE001 - reported to the parent
        err = type(e).__name__
    q.put((rank, err, log))
    q.close()
    q.join_thread()   # flush the put before a hard exit
    if rank == 1:
        # leave without further collectives: rank 0's pending all_reduce fails
        # once this process is gone instead of meeting a stray barrier
        os._exit(0)
    try:
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass


def test_two_ranks_one_raises():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, port, q)) for rk in range(2)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(2):
            rank, err, log = q.get(timeout=90)
            got[rank] = (err, log)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
                p.join()
    assert got[1][0] == "KeyError"
    # the raising rank never reached the barrier of the normal path
    assert got[1][1] == ["discard", "quiesce_local"]
    # its peer left its collective with an error instead of hanging
    assert got[0][0] is not None
    assert "quiesce" not in got[0][1]
