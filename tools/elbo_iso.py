"""ELBO-side kernels of one fit() iteration run alone on the GPU (no sweep
beside them), for rocprofv3 --kernel-trace --stats:

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/elbo_iso.py [--n N --T T --r R]

Launches ame_cov (covariance terms) and ame_elbo (pair + node + final kernels)
REPS times on the config-3 state after one sweep, synchronising between
launches, and prints the HIP-event average of each entry point."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--r", type=int, default=16)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    dev = torch.device("cuda", 0)
    m = TemporalAMEModel(a.n, a.T, a.r, seed=42)
    m.generate_data_fast(device=dev)
    vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=0.01, device=dev)
    vi.fit(max_iter=1, tolerance=0.0, verbose=False)
    eng = vi.engine
    torch.cuda.synchronize()
    eng.events.clear()
    eng.timing = True
    for _ in range(a.reps):
        eng.refresh_cov_terms()
        torch.cuda.synchronize()
        eng.launch_elbo()
        torch.cuda.synchronize()
    ms, _ = eng.kernel_ms()
    n, T, d = a.n, a.T, 2 + 2 * a.r
    print({"cov_ms": ms.get("cov"), "elbo_ms": ms.get("elbo"),
           "cov_GBs": 4.0 * n * T * d * d / (ms["cov"] * 1e-3) / 1e9,
           "pairs_alg_bytes": 4.0 * n * (n - 1) * T + 4.0 * n * T * 2 * a.r})


if __name__ == "__main__":
    main()
