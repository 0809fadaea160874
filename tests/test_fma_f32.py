"""fma_f32 (ame_amd.models.temporal_ame): an exact fp64 product plus an fp32
sum, rounded ONCE to fp32 -- the fused multiply-add the reference's fp32 sgemm /
2x2 matvec performs when it builds Y (temporal_ame.py:203-214, static_ame.py:216-236).
Checked against exact rational arithmetic, including the halfway cases where
rounding the fp64 sum to fp32 would round twice."""
from fractions import Fraction

import numpy as np
import torch

from ame_amd.models.temporal_ame import fma_f32


def _round_f32(x: Fraction) -> np.float32:
    """Round-to-nearest-even of an exact rational to fp32."""
    f = np.float32(float(x))
    best = None
    for c in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
        dist = abs(Fraction(float(c)) - x)
        key = (dist, int(np.array(c).view(np.uint32)) & 1)   # ties -> even mantissa
        if best is None or key < best[0]:
            best = (key, c)
    return best[1]


def _check(a, b, s):
    a, b, s = (np.asarray(v, np.float32) for v in (a, b, s))
    p = torch.from_numpy(a.astype(np.float64) * b.astype(np.float64))   # exact
    got = fma_f32(p, torch.from_numpy(s)).numpy()
    for k in range(a.size):
        want = _round_f32(Fraction(float(a.flat[k])) * Fraction(float(b.flat[k]))
                          + Fraction(float(s.flat[k])))
        assert got.flat[k] == want, (a.flat[k], b.flat[k], s.flat[k], got.flat[k], want)


def test_double_rounding_case():
    # s + a b = 1 + 3*2^-24 - 2^-54: the fp64 sum is the fp32 midpoint
    # 1 + 3*2^-24, whose ties-to-even rounding goes up; the true sum rounds down
    a = np.float32(2.0 ** -12 * (1 + 2.0 ** -15))
    b = np.float32(2.0 ** -12 * (1 - 2.0 ** -15))
    s = np.float32(1 + 2.0 ** -23)
    naive = np.float32(np.float64(a) * np.float64(b) + np.float64(s))
    _check([a], [b], [s])
    got = fma_f32(torch.tensor([float(a) * float(b)], dtype=torch.float64),
                  torch.tensor([s])).item()
    assert got == float(s) and float(naive) != float(s)


def test_random_against_exact():
    rng = np.random.default_rng(7)
    a = rng.standard_normal(3000).astype(np.float32)
    b = rng.standard_normal(3000).astype(np.float32)
    s = (rng.standard_normal(3000) * 4).astype(np.float32)
    _check(a, b, s)
