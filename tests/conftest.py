"""Shared pytest setup: import paths, the `gpu` marker, golden-fixture loaders."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "python-temporal-ame-svi_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libame_amd.so)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def golden_params(tag, dtype=np.float64):
    m = golden(f"{tag}_model.npz")
    return {k: m[k].astype(dtype) for k in ("R", "R_inv", "Sigma", "Psi", "Phi", "Q")}


@pytest.fixture
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
