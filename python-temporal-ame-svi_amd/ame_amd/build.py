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
SOURCES = ("ame_sweep.hip", "ame_sweep3.hip", "ame_cov.hip", "ame_elbo.hip", "ame_capi.hip",
           "ame_selftest.hip", "ame_align.hip", "ame_parts.hip")
# one-latent-dim diagnostic builds (-DAME_ONLY_R, tools/): no split parts, no router
UNSPLIT_SOURCES = tuple(s for s in SOURCES if s != "ame_parts.hip")
# Every latent dim 1..32 is compiled in; the heaviest sources are split into
# parts by r % parts (ame_common.h AME_R_PART) so the build runs in parallel.
SPLIT = {"ame_sweep.hip": 3, "ame_sweep3.hip": 2, "ame_elbo.hip": 2}


def _units():
    """(source, object, extra flags) for every translation unit."""
    out = []
    for src in SOURCES:
        parts = SPLIT.get(src, 1)
        for p in range(parts):
            if parts == 1:
                out.append((src, src.replace(".hip", ".o"), []))
            else:
                out.append((src, src.replace(".hip", f"_p{p}.o"), [f"-DAME_R_PART={p}", f"-DAME_R_NPART={parts}"]))
    return out
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
    units = _units()
    objs = [os.path.join(bdir, o) for _, o, _ in units]
    if not force and not _stale(objs):
        return OUT
    flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-pass-failed"]

    def compile_one(unit):
        src, obj, extra = unit
        cmd = [hipcc, *flags, *extra, "-c", os.path.join(CSRC, src), "-o", os.path.join(bdir, obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src} {extra}:\n{r.stderr[-4000:]}")
        return obj

    jobs = min(len(units), max(1, min(16, os.cpu_count() or 1)))
    # longest units first, so the tail of the parallel build is short
    order = sorted(units, key=lambda u: -{"ame_sweep.hip": 5, "ame_elbo.hip": 4, "ame_align.hip": 3,
                                          "ame_sweep3.hip": 2}.get(u[0], 1))
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, order))
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
