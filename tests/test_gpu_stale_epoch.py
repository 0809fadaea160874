"""Pipelined sweeps against stale hand-off words (verdict r04 item 1).

A pipelined sweep (epoch e + 1) starts on its own stream and waits ON THE
DEVICE until the previous sweep has flagged slices t and t+1 done (done[t] =
e).  Two conditions make that wait unsafe: the done array holds words from an
earlier use of the memory, and the host-issued zero fill that clears them has
not landed yet.  The test builds exactly that state, deterministically:

* the engine's own done flags are poisoned with an epoch far above any epoch
  this engine will use, the fill is made visible, then the MAIN stream is held
  busy by a long spin kernel and the zero fill + ``_mark_host_writes`` are
  queued behind it -- the pipelined launches of the next fit() are issued
  while the zero fill is still pending;
* with the engine's ordering (every pipelined launch waits for the event
  recorded after host writes) the fit is bit-equal to the in-order schedule;
* with that wait bypassed (test hook ``_order_after_host_writes = False``) the
  pipelined sweep meets the poisoned flags: the device's epoch-window check
  sets AME_STATUS_STALE_EPOCH and fit() raises instead of returning results
  computed from inputs that were never written.

Reference: structured_mf.py:211-287 (the Gauss-Seidel order the hand-offs
preserve).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPE = (128, 8, 4)      # n, T, r: v3, pipelined (2 * T_local fits on the chip)
POISON = 0x40000000      # far above any epoch a test process reaches


def _vi(opts):
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    n, T, r = SHAPE
    m = TemporalAMEModel(n, T, r, seed=5)
    m.generate_data_fast(seed=6)
    return TemporalAMEStructuredMFVI(m, learning_rate=0.5, device=torch.device("cuda", 0),
                                     engine_options=opts)


def _hold_main_stream(stream, ms=300.0):
    """Queue ~ms of spinning on `stream` (torch's spin kernel, clock64 based;
    the cycle count is calibrated once on this device)."""
    with torch.cuda.stream(stream):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        torch.cuda._sleep(1_000_000)
        b.record()
        b.synchronize()
        per_cycle = a.elapsed_time(b) / 1_000_000
        torch.cuda._sleep(int(ms / max(per_cycle, 1e-9)))


def _poisoned_pending_zero(eng):
    eng.done.fill_(POISON)
    torch.cuda.synchronize()
    _hold_main_stream(eng.stream)
    eng.done.zero_()                  # lands only after the spin
    eng._mark_host_writes()


def test_pipelined_launch_waits_for_pending_host_writes(gpu_device):
    ref = _vi({"speculate": False})
    ref.fit(max_iter=3, tolerance=0.0, verbose=False)
    want_m, want_c = ref.X_mean.numpy().copy(), ref.X_cov.numpy().copy()
    del ref
    vi = _vi(None)
    eng = vi.engine
    assert eng.pipelined and eng.spec_depth >= 2
    torch.cuda.synchronize()
    _poisoned_pending_zero(eng)
    vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    assert np.array_equal(vi.X_mean.numpy(), want_m)
    assert np.array_equal(vi.X_cov.numpy(), want_c)


def test_stale_done_flag_is_reported_not_consumed(gpu_device):
    vi = _vi(None)
    eng = vi.engine
    assert eng.pipelined
    torch.cuda.synchronize()
    eng._order_after_host_writes = False     # the hole the engine closes
    _poisoned_pending_zero(eng)
    try:
        with pytest.raises(RuntimeError, match="epoch outside the protocol") as ei:
            vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    finally:
        torch.cuda.synchronize()
    # the status block's record (include/ame_amd.h): one bit -- the waits behind
    # the first failure gave up quietly -- and the first wait's site, the
    # poisoned word it saw and the epoch it waited for
    w = [x & 0xFFFFFFFF for x in eng.last_status]
    print(str(ei.value))
    assert w[0] == 8, w                       # AME_STATUS_STALE_EPOCH only
    assert w[1] == 1 and w[2] in (1, 2), w    # done flag of slice t / t+1
    assert w[5] == POISON and 1 <= w[6] < POISON and w[8] == w[6] + 1, w
    assert 0 <= w[3] < SHAPE[1] and w[4] == 0xFFFFFFFF, w   # a slice, in the prologue
    assert "first failure: done flag of slice" in str(ei.value)


def test_process_epochs_increase_across_engines(gpu_device):
    """A second engine's epochs start above the first one's, so done flags or
    granules recycled from the first engine are below every epoch the second
    waits for (they make a waiter wait; they can never pass as current)."""
    a = _vi(None)
    a.fit(max_iter=2, tolerance=0.0, verbose=False)
    ea = a.engine.epoch
    b = _vi(None)
    eng = b.engine
    assert eng.epoch >= ea
    b.fit(max_iter=2, tolerance=0.0, verbose=False)
    assert eng.epoch > ea
