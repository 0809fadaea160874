"""CPU: the alignment restatement in oracle/ame_oracle.py against the reference's
own outputs (tests/golden/*_align.npz, written by make_golden_align.py from
src/utils/alignment.py).  The reference computes in fp32, the oracle in fp64:
agreement within 2e-5 * max(1, |x|)."""
import numpy as np
import pytest

import ame_oracle as O
from conftest import golden


@pytest.mark.parametrize("tag", ["c1", "mid", "wide"])
def test_alignment_oracle_vs_reference(tag):
    z = golden(f"{tag}_align.npz")
    r = int(z["r"])
    Xt = z["X_true"].astype(np.float64)
    for name in [k[:-4] for k in z.files if k.endswith("_est")]:
        Xe = z[f"{name}_est"].astype(np.float64)
        tol = 2e-5 * max(1.0, np.abs(Xt).max())
        each = O.align_temporal_states(Xe, Xt, r, True)
        assert np.abs(each - z[f"{name}_each"]).max() <= tol, name
        glob = O.align_temporal_states(Xe, Xt, r, False)
        assert np.abs(glob - z[f"{name}_global"]).max() <= tol, name
        err, _ = O.compute_alignment_error(Xe, Xt, r)
        assert abs(err - z[f"{name}_err"]) <= 1e-5 * z[f"{name}_err"]
        err0, _ = O.compute_alignment_error(Xe, Xt, r, align=False)
        assert abs(err0 - z[f"{name}_err_noalign"]) <= 1e-5 * z[f"{name}_err_noalign"]
        assert abs(O.correlation_after_alignment(Xe, Xt, r) - z[f"{name}_corr"]) <= 1e-6


def test_alignment_of_truth_is_identity():
    """Property: X_true^T X_true is symmetric PSD, so R = U Vt = I and every row
    keeps its sign -- aligning the truth to itself returns it unchanged."""
    rng = np.random.default_rng(3)
    Xt = rng.standard_normal((30, 4, 8))
    for each in (True, False):
        assert np.abs(O.align_temporal_states(Xt, Xt, 3, each) - Xt).max() < 1e-12
    assert O.compute_alignment_error(Xt, Xt, 3)[0] < 1e-24
