"""CPU: host-side pieces of ame_amd.utils (no kernels): the single-matrix
Procrustes / sign helpers against the oracle restatement, the reference's
compare_methods report, and the loud failure of the kernel path without a GPU."""
import numpy as np
import pytest
import torch

import ame_oracle as O


def test_procrustes_and_signs_match_oracle():
    from ame_amd.utils import align_signs, procrustes_alignment
    rng = np.random.default_rng(0)
    Xt = rng.standard_normal((40, 5))
    q, _ = np.linalg.qr(rng.standard_normal((5, 5)))
    Xe = Xt @ q + 0.01 * rng.standard_normal((40, 5))
    got, R = procrustes_alignment(torch.from_numpy(Xe), torch.from_numpy(Xt))
    ref, Rr = O.procrustes_alignment(Xe, Xt)
    assert np.allclose(R.numpy(), Rr, atol=1e-12) and np.allclose(got.numpy(), ref, atol=1e-12)
    flips = rng.random(40) < 0.5
    Xs = np.where(flips[:, None], -Xt, Xt) + 0.01 * rng.standard_normal(Xt.shape)
    out = align_signs(torch.from_numpy(Xs), torch.from_numpy(Xt), dim=1)
    assert np.array_equal(out.numpy(), O.align_signs_rows(Xs, Xt))
    # scaling option (alignment.py:93-98): a scaled copy is recovered exactly
    sc, _ = procrustes_alignment(torch.from_numpy(2.0 * Xt), torch.from_numpy(Xt), scaling=True)
    assert np.allclose(sc.numpy(), Xt, atol=1e-12)


def test_compare_methods_report(capsys):
    from ame_amd.utils import compare_methods, compute_state_prediction_error
    X = torch.zeros(3, 2, 6)
    res = {"Naive MF": {"history": {"reconstruction_error": [2.0, 1.0]}, "X_est": X + 1.0},
           "Good SMF": {"history": {"reconstruction_error": [2.0, 0.5]}, "X_est": X + 0.5}}
    compare_methods(res, metric="reconstruction_error", X_true=X)
    out = capsys.readouterr().out
    assert "1. Good SMF" in out and "2. Naive MF" in out
    assert "Improvement over Naive MF" in out and "+50.0%" in out
    assert compute_state_prediction_error(X, X + 0.5) == pytest.approx(0.25)


def test_alignment_kernel_path_needs_gpu():
    from ame_amd.utils import align_temporal_states
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    X = torch.zeros(4, 2, 6)
    with pytest.raises(RuntimeError):
        align_temporal_states(X, X, 2)


def test_run_method_with_timing_contract(capsys):
    """experiments/utils.py:146-229 result keys and prints, on a host-only VI
    stand-in (the device engine's kernel times are added when it has one)."""
    from ame_amd.utils import run_method_with_timing

    class FakeVI:
        def __init__(self, model, learning_rate=1.0):
            self.model, self.lr = model, learning_rate
            self.X_mean = torch.ones(2, 3, 4)

        def fit(self, max_iter=100, verbose=True):
            return {"elbo": [torch.tensor(-3.0)] * max_iter,
                    "reconstruction_error": [0.5] * max_iter}

    res = run_method_with_timing(FakeVI, object(), "Fake", max_iter=4, learning_rate=0.1)
    assert res["iterations"] == 4 and res["method_name"] == "Fake"
    assert res["vi"].lr == 0.1 and torch.equal(res["X_est"], torch.ones(2, 3, 4))
    assert res["runtime"] >= 0 and "kernels_ms" not in res
    out = capsys.readouterr().out
    assert "Running: Fake" in out and "Final MSE: 0.500000" in out
