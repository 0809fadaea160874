"""Hand-off waits behind a late rank, and the CU co-residency edge (GPU).

* A time-sharded run in which one rank reaches its first sweep 3 s after the
  other (host jitter, a slow first collective): two ranks on one GPU at config
  4's per-rank shape (n=1024, T_local=64, r=16).  The late rank's neighbour
  waits on the halo / back channel (10 s budget) and its other slices wait
  behind that on this GPU; under the round-6 wait rules (include/ame_amd.h
  status block) those local waits restart their 2 s budget while a cross-rank
  wait is in flight, so no status is raised and the fit is bit-equal to one
  process.  Before round 6 the local waits timed out after 2 s
  (profiles/r05_fin6_pytest_gpu_fail.txt had that shape of failure).
* Config 3's pipelined fit while a foreign kernel holds part of the chip: the
  result is bit-equal to the undisturbed fit or fit() raises a device status
  with its first-failure record -- never a silent difference.

Reference: structured_mf.py:240-287 (the node / time order the hand-offs keep).
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _vi(model, dev, distributed=None, **opts):
    from ame_amd import TemporalAMEStructuredMFVI
    return TemporalAMEStructuredMFVI(model, factorization="good", learning_rate=0.01, device=dev,
                                     distributed=distributed, engine_options=opts)


def _model(dev, n=1024, T=128, r=16):
    from ame_amd import TemporalAMEModel
    m = TemporalAMEModel(n, T, r, seed=42)
    m.generate_data_fast(device=dev, seed=42)
    return m


def _run(distributed, delay_rank=-1, delay_s=0.0):
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    vi = _vi(_model(dev), dev, distributed=distributed)
    e = vi.engine
    rank = dist.get_rank() if distributed else 0
    if rank == delay_rank:
        e._first_launch_delay_s = delay_s
    h = vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    status = e.status.cpu().tolist()
    mean = vi.X_mean.numpy().copy()
    digest = hashlib.sha256(vi.X_cov.numpy().tobytes()).hexdigest()
    return (mean, digest, [float(x) for x in h["elbo"]], list(h["reconstruction_error"]), status,
            (e.device_sharers, e.coresident_launches, max(sz for _, sz in e.groups), e.resident_slots,
             e.pipelined))


def _worker(rank, world, port, delay_rank, delay_s, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = _run(True, delay_rank, delay_s)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("delay_rank", [0, 1])
def test_late_rank_is_exact(delay_rank, gpu_device):
    """One rank sleeps 3 s before its first sweep launch (after that sweep's
    collectives); rank 0 late: rank 1's first slice waits on the halo and its
    other 63 slices behind it; rank 1 late: rank 0's last slice of the next
    (pipelined) sweep waits on the back channel and the sweep after it behind
    that.  Both ranks finish without a status, bit-equal to one process."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, 2, port, delay_rank, 3.0, q)) for rk in range(2)]
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
    assert sorted(outs) == [0, 1]
    for rk in (0, 1):
        st = outs[rk][4]
        assert not any(st[:11]), f"rank {rk} status block {st}"
    # the waiting rank's first slice (halo) or last slice (back channel) spun for
    # about the delay, accounted in status words 11 / 12 (microseconds)
    waiter, word = (1, 11) if delay_rank == 0 else (0, 12)
    waited_ms = outs[waiter][4][word] / 1e3
    print(f"rank {delay_rank} late by 3 s: rank {waiter} cross-rank wait {waited_ms:.0f} ms "
          f"(status words 11/12: {outs[waiter][4][11:13]})")
    assert waited_ms > 1000.0, outs[waiter][4]
    for rk in (0, 1):
        sharers, launches, group, slots, pipelined = outs[rk][5]
        assert pipelined and sharers == 2 and sharers * launches * group <= slots
    mean_s, dig_s, elbo_s, rec_s, _, _ = _run(False)
    mean_d, dig_d, elbo_d, rec_d = outs[0][:4]
    assert np.array_equal(mean_d, mean_s)
    assert dig_d == dig_s
    assert np.allclose(elbo_d, elbo_s, rtol=1e-6, atol=0)
    assert np.allclose(rec_d, rec_s, rtol=1e-12, atol=0)


@pytest.mark.parametrize("cus,us", [(96, 1_200_000), (200, 1_200_000)])
def test_pipelined_fit_beside_cu_hog(cus, us, gpu_device):
    """Config 3's production fit (two pipelined 128-slice launches = every CU)
    started while `cus` one-per-CU workgroups of a foreign kernel hold their
    CUs for `us` microseconds on another stream.  The sweep's workgroups then
    cannot all be resident until the hog ends: the fit is bit-equal to the
    undisturbed one, or fit() raises the device status (never a silent
    difference)."""
    import ame_amd._lib as L
    dev = gpu_device
    ref = _vi(_model(dev), dev)
    ref.fit(max_iter=3, tolerance=0.0, verbose=False)
    ref_mean = ref.X_mean.numpy().copy()
    ref_dig = hashlib.sha256(ref.X_cov.numpy().tobytes()).hexdigest()
    del ref
    torch.cuda.empty_cache()
    vi = _vi(_model(dev), dev)
    assert vi.engine.pipelined
    lib = L.lib()
    touched = torch.zeros(1, dtype=torch.int32, device=dev)
    hog = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize(dev)
    rc = lib.ame_debug_occupy(int(cus), 160 * 1024, int(us), ctypes_ptr(touched), ctypes_stream(hog))
    assert rc == 0
    try:
        vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    except RuntimeError as exc:
        # a raised status names its first failing wait
        msg = str(exc)
        print(f"hog {cus} CUs: fit raised: {msg}")
        assert "device status" in msg and "first failure" in msg, msg
        torch.cuda.synchronize(dev)
        return
    torch.cuda.synchronize(dev)
    assert int(touched.item()) == 1
    print(f"hog {cus} CUs x {us / 1e6:.1f} s: fit completed; comparing with the undisturbed fit")
    assert np.array_equal(vi.X_mean.numpy(), ref_mean)
    assert hashlib.sha256(vi.X_cov.numpy().tobytes()).hexdigest() == ref_dig
    assert not any(vi.engine.status.cpu().tolist())


def ctypes_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


def ctypes_stream(s):
    import ctypes
    return ctypes.c_void_p(s.cuda_stream)


def test_starved_sweep_raises_one_record(gpu_device):
    """The other side of the co-residency edge: a foreign kernel holds 200 CUs
    for 3.5 s, longer than the 2 s local budget, while config 3's 128-slice
    sweep starts.  The slices that did get a CU wait on neighbours that did not;
    the first wait to outlive its budget raises SPIN_TIMEOUT with its record,
    and every later wait gives up quietly -- one bit, one record, no second
    status manufactured by the first (include/ame_amd.h wait rules)."""
    import ame_amd._lib as L
    dev = gpu_device
    vi = _vi(_model(dev), dev)
    eng = vi.engine
    lib = L.lib()
    touched = torch.zeros(1, dtype=torch.int32, device=dev)
    hog = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize(dev)
    assert lib.ame_debug_occupy(200, 160 * 1024, 3_500_000, ctypes_ptr(touched), ctypes_stream(hog)) == 0
    with pytest.raises(RuntimeError) as ei:
        vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    torch.cuda.synchronize(dev)
    msg = str(ei.value)
    print(msg)
    w = [x & 0xFFFFFFFF for x in eng.last_status]
    # one bit: the slice-to-slice wait (or, if a helper's spin outlasts the
    # solver's, the LDS counter behind it) -- never both
    assert w[0] in (L.AME_STATUS_SPIN_TIMEOUT, L.AME_STATUS_LDS_TIMEOUT), w
    assert w[1] == 1 and w[2] in L.AME_WAIT_SITES and w[7] >= 2_000_000, w
    assert "first failure:" in msg
