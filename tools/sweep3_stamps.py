"""Diagnostic for the v3 sweep (ame_sweep3.hip): in-kernel s_memtime stamps.

    python tools/sweep3_stamps.py --build      # here: hipcc -DAME_STAMPS -> tools/_lib/libame_amd_stamps3.so
    python tools/sweep3_stamps.py [--tag=T] [--iters=K]   # GPU box: config-3 fit, per-wave timelines
                                               # of the last sweep (K > 2: a pipelined steady-state one)

The stamped build's run time is never quoted; only its shares / timelines.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "python-temporal-ame-svi_amd")
BDIR = os.path.join(PKG, "ame_amd", "_build")      # objects (not shipped to the GPU box)
LIBDIR = os.path.join(ROOT, "tools", "_lib")         # variant libraries (shipped)
TAG = ([a.split("=", 1)[1] for a in sys.argv if a.startswith("--tag=")] or [""])[0]
SO = os.path.join(LIBDIR, f"libame_amd_stamps3{TAG}.so")

def _unsplit_sources():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "python-temporal-ame-svi_amd"))
    from ame_amd.build import UNSPLIT_SOURCES
    return UNSPLIT_SOURCES

NAMES = {   # stamp slot names per wave (the kernel stamps every wave; see ame_sweep3.hip STAMP3)
    0: ["start", "J+kj", "reduce", "(was: HX wait)", "2x2+assembly", "publish", "kcnt", "brow", "gcnt", "prep(v,yv)"],
}
for _w in range(1, 8):
    _hw = _w - 1
    NAMES[_w] = ["start",
                 "pring" if _hw <= 2 else "-",
                 "poll" if _hw <= 2 else "-",
                 "hf1" if _hw <= 2 else "-",
                 "HB" if _hw <= 5 else "(no HB)",
                 "GEMV",
                 "DMA" if _hw == 6 else ("spin" if _hw <= 2 else "-"),
                 "gemv-fma", "gemv-rs",
                 "vmwait" if _hw == 6 else "end",
                 "pre-pring"]
WAVES = ["solver(w0)"] + [f"hw{w - 1}(w{w})" for w in range(1, 8)]


def build(r=16):
    os.makedirs(BDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    csrc = os.path.join(PKG, "ame_amd", "csrc")
    defs = [f"-D{d}" for d in (" ".join(a for a in sys.argv if a.startswith("--defs=")).replace(
        "--defs=", "")).split(",") if d]
    objs = []
    for src in _unsplit_sources():
        o = os.path.join(BDIR, src.replace(".hip", f"_s3{TAG}.o"))
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                               "-std=c++17", "-DAME_STAMPS", f"-DAME_ONLY_R={r}", *defs,
                               "-Wno-pass-failed", "-c", os.path.join(csrc, src), "-o", o])
        objs.append(o)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC",
                           "-o", SO, *objs])
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
    iters = int(([a.split("=", 1)[1] for a in sys.argv if a.startswith("--iters=")] or ["2"])[0])
    vi.fit(max_iter=iters, tolerance=0.0, verbose=False)   # stamps: the last sweep that ran
    torch.cuda.synchronize()
    L = _lib.lib()
    L.ame_debug_read_stamps3.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    st = np.zeros(8 * 16 * 16, dtype=np.uint64)
    pg = np.zeros(256 * 5, dtype=np.uint64)
    assert L.ame_debug_read_stamps3(st.ctypes.data, pg.ctypes.data) == 0
    st = st.reshape(8, 16, 16).astype(np.int64)
    L.ame_debug_read_hwid3.argtypes = [ctypes.c_void_p]
    hw = np.zeros(8, dtype=np.uint32)
    L.ame_debug_read_hwid3(hw.ctypes.data)
    print("HW_ID per wave (wave_id, simd_id, cu_id):",
          [(int(h & 15), int((h >> 4) & 3), int((h >> 8) & 15)) for h in hw])
    pg = pg.reshape(256, 5).astype(np.int64)[:128]
    t0 = st[0, :, 0].min()
    print("step period (solver start-to-start), cycles:", np.diff(st[0, :, 0])[:15].tolist())
    for w in range(8):
        print(f"--- {WAVES[w]} (cycles after solver step start, median over 16 steps)")
        rel = st[w] - st[0, :, 0][:, None]
        for sl, nm in enumerate(NAMES[w]):
            if nm == "-" or st[w, :, sl].max() == 0:
                continue
            hit = st[w, :, sl] != 0
            print(f"  {sl:2d} {nm:14s} {int(np.median(rel[hit, sl])):8d}  ({int(hit.sum())}/16 steps)")
    pr = (pg - pg[:, :1]) / 100.0   # us (100 MHz realtime)
    st0 = (pg[:, 0] - pg[0, 0]) / 100.0
    print("lane start offset (us) at lanes 0,1,2,4,8,16,32,64,127:",
          [round(float(st0[k]), 1) for k in (0, 1, 2, 4, 8, 16, 32, 64, 127)])
    print("per-lane elapsed (us) to n/4, n/2, 3n/4, n; lanes 0, 64, 127:")
    for k in (0, 64, 127):
        print("  ", k, [round(float(x), 1) for x in pr[k, 1:]])


if __name__ == "__main__":
    build() if "--build" in sys.argv else run()
