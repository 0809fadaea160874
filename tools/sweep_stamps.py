"""Diagnostic: per-phase cycle shares of one sweep step (in-kernel s_memtime stamps).

    python tools/sweep_stamps.py --build      # here: hipcc -DAME_STAMPS -> _build/libame_amd_stamps.so
    python tools/sweep_stamps.py              # GPU box: config-3 sweep, print phase shares

Stamps are taken by thread 0 of the middle lane for 16 nodes in steady state.
The stamped build's run time is never quoted; only its SHARES are meaningful.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "python-temporal-ame-svi_amd")
BDIR = os.path.join(PKG, "ame_amd", "_build")
SO = os.path.join(BDIR, "libame_amd_stamps.so")
PHASES = ["snap+Yrow+vectors+poll", "GEMV+AR", "reduce+P build", "Gauss-Jordan",
          "mu out+granules", "stats update", "M update (+next step start)"]


def build(r=16):
    os.makedirs(BDIR, exist_ok=True)
    csrc = os.path.join(PKG, "ame_amd", "csrc")
    objs = []
    for src in ("ame_sweep.hip", "ame_cov.hip", "ame_elbo.hip", "ame_capi.hip"):
        o = os.path.join(BDIR, src.replace(".hip", "_stamps.o"))
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                               "-DAME_STAMPS", f"-DAME_ONLY_R={r}", "-Wno-pass-failed", "-c",
                               os.path.join(csrc, src), "-o", o])
        objs.append(o)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO, *objs])
    print("built", SO)


def run():
    os.environ["AME_LIB_PATH"] = SO
    sys.path.insert(0, PKG)
    import torch
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    from ame_amd import _lib
    dev = torch.device("cuda", 0)
    m = TemporalAMEModel(1024, 128, 16, seed=42)
    m.generate_data_fast(device=dev)
    vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=0.01, device=dev)
    vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    torch.cuda.synchronize()
    L = _lib.lib()
    L.ame_debug_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * (16 * 8))()
    assert L.ame_debug_read_stamps(buf, 16 * 8) == 0
    rows = [[buf[k * 8 + p] for p in range(8)] for k in range(16)]
    tot = [0.0] * 7
    step = []
    for k in range(15):
        r, nxt = rows[k], rows[k + 1]
        seq = r[:7] + [nxt[0]]
        for p in range(7):
            tot[p] += seq[p + 1] - seq[p]
        step.append(nxt[0] - r[0])
    T = sum(tot)
    print(f"mean step {sum(step) / len(step):.0f} cycles (s_memtime ticks)")
    for name, t in zip(PHASES, tot):
        print(f"  {name:32s} {t / 15:9.0f}  {100 * t / T:5.1f}%")


if __name__ == "__main__":
    build() if "--build" in sys.argv else run()
