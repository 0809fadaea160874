"""Build a one-latent-dim variant library for same-box A/B runs (tools/ab_v3.py).

    python tools/build_variant.py --r=16 --tag=X [--defs=A,B] [--flags=-f1,-f2]   -> tools/_lib/libame_amd_X.so

Unsplit sources, -DAME_ONLY_R=<r>, plus -D<def> for each listed switch.  A
variant library is a diagnostic: it is never the product build (build.py)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "python-temporal-ame-svi_amd")
BDIR = os.path.join(PKG, "ame_amd", "_build")
LIBDIR = os.path.join(ROOT, "tools", "_lib")


def _opt(name, default=None):
    for a in sys.argv:
        if a.startswith(name + "="):
            return a.split("=", 1)[1]
    return default


def main():
    sys.path.insert(0, PKG)
    from ame_amd.build import UNSPLIT_SOURCES
    r = int(_opt("--r", 16))
    tag = _opt("--tag", f"r{r}")
    defs = [f"-D{d}" for d in (_opt("--defs") or "").split(",") if d]
    defs += [f for f in (_opt("--flags") or "").split(",") if f]   # extra compiler flags
    os.makedirs(BDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    csrc = os.path.join(PKG, "ame_amd", "csrc")

    def one(src):
        o = os.path.join(BDIR, src.replace(".hip", f"_var_{tag}.o"))
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                               f"-DAME_ONLY_R={r}", *defs, "-Wno-pass-failed",
                               "-c", os.path.join(csrc, src), "-o", o])
        return o

    with ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(one, UNSPLIT_SOURCES))
    so = os.path.join(LIBDIR, f"libame_amd_{tag}.so")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", so, *objs])
    print("built", so)


if __name__ == "__main__":
    main()
