"""Build libame_amd.so in-tree with hipcc for gfx950 (no torch extension, no JIT cache).

    python -m ame_amd.build            # from python-temporal-ame-svi_amd/
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libame_amd.so")
SOURCES = ("ame_sweep.hip", "ame_sweep3.hip", "ame_sweep4.hip", "ame_cov.hip", "ame_elbo.hip", "ame_capi.hip",
           "ame_selftest.hip", "ame_align.hip")
ARCH = os.environ.get("AME_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build ame_amd)")


def _stale(objs):
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(HERE, "..", "..", "include", "ame_amd.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> str:
    hipcc = _hipcc()
    bdir = os.path.join(HERE, "_build")
    os.makedirs(bdir, exist_ok=True)
    objs = [os.path.join(bdir, s.replace(".hip", ".o")) for s in SOURCES]
    if not force and not _stale(objs):
        return OUT
    flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-pass-failed"]

    def compile_one(src, obj):
        cmd = [hipcc, *flags, "-c", os.path.join(CSRC, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-4000:]}")
        return obj

    jobs = min(len(SOURCES), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda so: compile_one(*so), zip(SOURCES, objs)))
    tmp = OUT + ".tmp"
    r = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, OUT)
    if verbose:
        print(f"built {OUT}", file=sys.stderr)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
