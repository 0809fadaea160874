"""Build libame_amd.so in-tree with hipcc for gfx950 (no torch extension, no JIT cache).

    python -m ame_amd.build            # from python-temporal-ame-svi_amd/
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import re
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


FLAGS = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-pass-failed"]
_VERSION_RE = re.compile(rb"ame_amd 0\.\d+ gfx950 src=([0-9a-f]{16}|unknown)")


def _inputs():
    """Every file the library is built from: csrc/* and the C-ABI header."""
    files = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                   if f.endswith((".hip", ".h")))
    files.append(os.path.join(HERE, "..", "..", "include", "ame_amd.h"))
    return [f for f in files if os.path.exists(f)]


def source_hash() -> str:
    """SHA-256 prefix over the sources, headers, flags and split layout: what
    ame_version() of a library built from this tree reports after "src="."""
    h = hashlib.sha256()
    h.update(repr((FLAGS, sorted(SPLIT.items()), SOURCES)).encode())
    for f in _inputs():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def embedded_hash(path: str = OUT):
    """The src= hash compiled into a built library (read from the file, not
    loaded), or None."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        m = _VERSION_RE.search(fh.read())
    return m.group(1).decode() if m else None


def _unit_key(src, extra, headers_digest, src_hash):
    h = hashlib.sha256()
    with open(os.path.join(CSRC, src), "rb") as fh:
        h.update(fh.read())
    h.update(headers_digest.encode())
    h.update(repr((FLAGS, extra)).encode())
    if src == "ame_capi.hip":
        h.update(src_hash.encode())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = True) -> str:
    """Rebuild when the library's embedded source hash differs from the tree's
    (content, not mtimes); objects whose inputs did not change are reused."""
    src_hash = source_hash()
    if not force and embedded_hash(OUT) == src_hash:
        return OUT
    hipcc = _hipcc()
    bdir = os.path.join(HERE, "_build")
    os.makedirs(bdir, exist_ok=True)
    units = _units()
    objs = [os.path.join(bdir, o) for _, o, _ in units]
    hd = hashlib.sha256()
    for f in _inputs():
        if f.endswith(".h"):
            with open(f, "rb") as fh:
                hd.update(fh.read())
    headers_digest = hd.hexdigest()

    def compile_one(unit):
        src, obj, extra = unit
        if src == "ame_capi.hip":
            extra = [*extra, f'-DAME_SRC_HASH="{src_hash}"']
        key = _unit_key(src, extra, headers_digest, src_hash)
        opath = os.path.join(bdir, obj)
        kpath = opath + ".key"
        if not force and os.path.exists(opath) and os.path.exists(kpath) \
                and open(kpath).read() == key:
            return obj
        cmd = [hipcc, *FLAGS, *extra, "-c", os.path.join(CSRC, src), "-o", opath]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src} {extra}:\n{r.stderr[-4000:]}")
        with open(kpath, "w") as fh:
            fh.write(key)
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
    got = embedded_hash(tmp)
    if got != src_hash:
        raise RuntimeError(f"built library reports src={got}, tree is {src_hash}")
    os.replace(tmp, OUT)
    if verbose:
        print(f"built {OUT} (src={src_hash})", file=sys.stderr)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
