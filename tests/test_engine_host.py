"""Host-side engine logic (no GPU): explicit options, the queue-depth model,
slice groups.  DESIGN.md §5."""
import pytest

from ame_amd.engine import EngineOptions, derive_spec_depth, slice_groups


def test_options_are_explicit():
    o = EngineOptions.coerce(None)
    assert o == EngineOptions()
    assert EngineOptions.coerce({"spec_depth": 3}).spec_depth == 3
    assert EngineOptions.coerce(o) is o
    with pytest.raises(ValueError, match="unknown engine option"):
        EngineOptions.coerce({"spec_dpeth": 3})
    # the ELBO-beside-the-sweep split is opt-in (0: off; the engine checks the
    # kernel and the CU count when it is built, tests/test_gpu_w6_workers.py)
    assert EngineOptions().elbo_cus == 0
    assert EngineOptions.coerce({"elbo_cus": 32, "sweep_kernel": 24}).elbo_cus == 32
    # ELBO-before-the-speculative-sweep: opt-in, measured no faster
    # (tests/test_gpu_w6_workers.py::test_elbo_first_bit_equal)
    assert EngineOptions().elbo_first is False
    assert EngineOptions.coerce({"elbo_first": True}).elbo_first is True


def test_queue_depth_model():
    """(1 + depth) P >= fill + C + delta with P ~ C = n steps."""
    # config 3 on one GPU and the weak-scaling series (T = 128 per GPU)
    assert derive_spec_depth(1024, 128) == 2
    assert derive_spec_depth(1024, 256) == 2
    assert derive_spec_depth(1024, 512) == 2
    assert derive_spec_depth(1024, 1024) == 4      # N = 8: fill 3.0 x 1023 steps > 3 chains
    # the model's margin at N = 8 and depth 4: (1 + 4) n >= 3.0 (T - 1) + n + 128
    n, T = 1024, 1024
    assert (1 + 4) * n >= 3.0 * (T - 1) + n + 128
    assert (1 + 3) * n < 3.0 * (T - 1) + n + 128   # depth 3 would stall (by ~1 %)
    # short chains, many slices: deeper, capped
    assert derive_spec_depth(256, 512) == 7
    assert derive_spec_depth(16, 4096) == 8
    assert derive_spec_depth(4096, 32) == 2


def test_slice_groups_cover_in_order():
    for T, cap, force in [(512, 256, 0), (10, 256, 3), (7, 7, 0), (300, 128, 0), (5, 256, 128)]:
        g = slice_groups(T, cap, force)
        assert sum(sz for _, sz in g) == T
        assert all(b[0] == a[0] + a[1] for a, b in zip(g, g[1:]))
        assert max(sz for _, sz in g) <= (cap if force <= 0 else min(force, cap))
    with pytest.raises(RuntimeError):
        slice_groups(4, 0)


def test_status_report_names_the_first_failure():
    """The status block (include/ame_amd.h AME_STATUS_WORDS): bits, the first
    failing wait's record, and the count of waits that gave up behind it."""
    from ame_amd import _lib
    from ame_amd.engine import status_report
    assert _lib.AME_STATUS_WORDS == 16
    w = [0] * 16
    w[0] = _lib.AME_STATUS_SPIN_TIMEOUT
    w[1], w[2], w[3], w[4], w[5], w[6], w[7], w[8] = 1, 4, 65, 17, 6, 7, 2_000_123, 7
    w[10] = 12
    msg = status_report(w)
    assert msg.startswith("device status 0x1: a hand-off between slices timed out")
    assert "first failure: hand-off granule of slice t-1, slice 65, node 17, saw 6 expected 7" in msg
    assert "after 2000.1 ms, sweep epoch 7" in msg and "12 later wait(s) gave up quietly" in msg
    w2 = [_lib.AME_STATUS_STALE_EPOCH, 1, 2, 3, 0xFFFFFFFF, 9, 4, 0, 5] + [0] * 7
    assert "done flag of slice t+1 (previous sweep), slice 3, prologue, saw 9 expected 4" in status_report(w2)
    # negative int32 words from the device tensor are read as uint32
    w3 = [8, 1, 3, 0, -1, -2, 5, 0, 6] + [0] * 7
    assert "prologue, saw 4294967294 expected 5" in status_report(w3)
