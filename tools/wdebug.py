"""Debug build of the v2 GEMV-worker sweep (printf on spin timeouts).
   python tools/wdebug.py --build   (here)     python tools/wdebug.py  (GPU box)"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "python-temporal-ame-svi_amd")
BDIR = os.path.join(PKG, "ame_amd", "_build")      # objects (not shipped to the GPU box)
LIBDIR = os.path.join(ROOT, "tools", "_lib")         # variant libraries (shipped)
SO = os.path.join(LIBDIR, "libame_amd_wdbg.so")

def _unsplit_sources():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "python-temporal-ame-svi_amd"))
    from ame_amd.build import UNSPLIT_SOURCES
    return UNSPLIT_SOURCES

if "--build" in sys.argv:
    os.makedirs(BDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    objs = []
    for src in _unsplit_sources():
        o = os.path.join(BDIR, src.replace(".hip", "_wd.o"))
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                               "-DAME_WDEBUG", "-DAME_ONLY_R=32", "-Wno-pass-failed", "-c",
                               os.path.join(PKG, "ame_amd", "csrc", src), "-o", o])
        objs.append(o)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO, *objs])
    print("built", SO)
else:
    os.environ["AME_LIB_PATH"] = SO
    sys.path.insert(0, PKG)
    import torch
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    dev = torch.device("cuda", 0)
    for (n, T) in ((24, 1), (24, 3)):
        m = TemporalAMEModel(n, T, 32, seed=7)
        m.generate_data_fast(seed=11)
        vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=0.5, device=dev)
        print("kind", vi.engine.sweep_kind, flush=True)
        try:
            vi.fit(max_iter=1, tolerance=0.0, verbose=False)
            print(n, T, "ok", flush=True)
        except RuntimeError as e:
            print(n, T, "ERR", e, flush=True)
        torch.cuda.synchronize()
