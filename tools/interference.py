"""Does the ELBO side (covariance-terms + ELBO kernels, run beside the pipelined
sweeps) slow the sweep down?  Config 3 by default, one GPU:

    [AME_VAR_R=32] python tools/interference.py --build TAG DEF1,DEF2   # here: variant library tools/_lib/libame_amd_var{TAG}.so (r = 16 unless AME_VAR_R)
    python tools/interference.py [--shape n,T,r] [TAG ...]   # GPU box: per library, fit vs sweeps-only

(A) ms per fit() iteration (the bench's loop); (B) ms per sweep when the same
pipelined, two-deep sweep queue runs with no ELBO side at all.  Diagnostic
only: (B) skips the ELBO, so it is never a bench number."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "python-temporal-ame-svi_amd")
BDIR = os.path.join(PKG, "ame_amd", "_build")      # objects (not shipped to the GPU box)
LIBDIR = os.path.join(ROOT, "tools", "_lib")         # variant libraries (shipped)

def _unsplit_sources():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "python-temporal-ame-svi_amd"))
    from ame_amd.build import UNSPLIT_SOURCES
    return UNSPLIT_SOURCES



def build(tag, defs):
    os.makedirs(BDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    csrc = os.path.join(PKG, "ame_amd", "csrc")
    objs = []
    procs = []
    for src in _unsplit_sources():
        o = os.path.join(BDIR, src.replace(".hip", f"_var{tag}.o"))
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                                       f"-DAME_ONLY_R={os.environ.get('AME_VAR_R', '16')}",
                                       *[f"-D{d}" for d in defs if d], "-Wno-pass-failed",
                                       "-c", os.path.join(csrc, src), "-o", o]))
        objs.append(o)
    for p in procs:
        assert p.wait() == 0
    so = os.path.join(LIBDIR, f"libame_amd_var{tag}.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", so, *objs])
    print("built", so)


def measure(K=20, shape=(1024, 128, 16)):
    sys.path.insert(0, PKG)
    import torch
    from ame_amd import TemporalAMEModel, TemporalAMEStructuredMFVI
    dev = torch.device("cuda", 0)
    m = TemporalAMEModel(*shape, seed=42)
    m.generate_data_fast(device=dev)
    vi = TemporalAMEStructuredMFVI(m, factorization="good", learning_rate=0.01, device=dev)
    vi.fit(max_iter=3, tolerance=0.0, verbose=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vi.fit(max_iter=K, tolerance=0.0, verbose=False)
    torch.cuda.synchronize()
    fit_ms = (time.perf_counter() - t0) * 1e3 / K
    eng = vi.engine
    eng.discard_speculation()
    torch.cuda.synchronize()
    res = {}
    for label, depth in (("sweeps_only", 2),):
        for _ in range(3):
            eng.speculate(depth)
            eng.sweep()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            eng.speculate(depth)
            eng.sweep()
        eng.discard_speculation()
        torch.cuda.synchronize()
        res[label] = (time.perf_counter() - t0) * 1e3 / K
    eng._check_status()
    return {"shape": list(shape), "sweep_kind": int(eng.sweep_kind), "pipelined": bool(eng.pipelined),
            "fit_ms_per_iter": fit_ms, **{k + "_ms": v for k, v in res.items()},
            "lib": os.environ.get("AME_LIB_PATH", "default")}


if __name__ == "__main__":
    if "--build" in sys.argv:
        k = sys.argv.index("--build")
        build(sys.argv[k + 1], sys.argv[k + 2].split(",") if len(sys.argv) > k + 2 else [])
    elif "--child" in sys.argv:
        shape = tuple(int(x) for x in sys.argv[sys.argv.index("--child") + 1].split(","))
        K = 20 if shape[0] <= 1024 else 8
        print(json.dumps(measure(K, shape)))
    else:
        args = sys.argv[1:]
        shape = "1024,128,16"
        if "--shape" in args:
            k = args.index("--shape")
            shape = args[k + 1]
            del args[k:k + 2]
        for tag in ["default"] + args:
            env = dict(os.environ)
            if tag != "default":
                env["AME_LIB_PATH"] = os.path.join(LIBDIR, f"libame_amd_var{tag}.so")
            for rep in range(2):
                r = subprocess.run([sys.executable, "-u", __file__, "--child", shape], env=env, capture_output=True,
                                   text=True, timeout=300)
                if r.returncode != 0:
                    print(tag, "failed", r.stderr[-2000:])
                    sys.exit(1)
                print(tag, rep, r.stdout.strip().splitlines()[-1], flush=True)
