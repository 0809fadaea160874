"""Device self-test of the primitives the v3 sweep kernel is built on:
the 64-lane reduce-scatter (ame_wave.h) for fp32 and fp64 and LDS-DMA
(global_load_lds) placement.  Exact expected values (integer-valued sums)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_wave_reduce_scatter_and_dma(gpu_device):
    from ame_amd import _lib
    L = _lib.lib()
    src = torch.arange(1024, dtype=torch.float32, device=gpu_device) * 0.5
    out = torch.full((1024,), -1.0, dtype=torch.float32, device=gpu_device)
    rc = L.ame_debug_selftest(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(out.data_ptr()))
    assert rc == 0
    o = out.cpu().numpy()
    lanes = np.arange(64)
    # fp32, 34 values: v[q] = 3*lane + q  -> sum_q = 3*2016 + 64 q
    idx, val = o[:64].astype(int), o[64:128]
    seen = {}
    for i, v in zip(idx, val):
        if i < 34:
            assert i not in seen, f"index {i} owned twice"
            seen[i] = v
    assert sorted(seen) == list(range(34))
    for q, v in seen.items():
        assert v == 3 * lanes.sum() + 64 * q, (q, v)
    # fp64, 20 values: v[q] = 5*lane + q + 0.25
    idx, val = o[128:192].astype(int), o[192:256]
    seen = {}
    for i, v in zip(idx, val):
        if i < 20:
            assert i not in seen
            seen[i] = v
    assert sorted(seen) == list(range(20))
    for q, v in seen.items():
        assert v == 5 * lanes.sum() + 64 * q + 16.0, (q, v)
    s = src.cpu().numpy()
    assert np.array_equal(o[256:512], s[:256])
    assert np.array_equal(o[512:768], s[256:512])
    assert np.array_equal(o[768:832], s[600:664])
