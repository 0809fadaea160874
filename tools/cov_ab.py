"""A/B of the covariance-terms kernel (K2, ame_cov) on one box, isolated launches.

    python tools/cov_ab.py LIB_A LIB_B ... [--shapes n,T,r;n,T,r] [--rounds 3] [--reps 20]

Each (library, shape) runs in its own process with AME_LIB_PATH set: random
SPD fp32 covariances of the shape on the GPU (slice 0 included: t_begin 0),
ame_cov launched REPS times after 3 warmup launches, HIP events on the launch
stream; prints ms per launch and the HBM fraction of its algorithmic bytes
(4 n T d^2).  Libraries alternate round-robin, so box drift hits both."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(n, T, r, reps):
    sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))
    import torch
    from ame_amd import _lib
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    d = 2 + 2 * r
    g = torch.Generator(device=dev).manual_seed(1)
    cov = torch.empty(T * n, d, d, device=dev)
    for s in range(0, T * n, 8192):
        X = torch.randn(min(8192, T * n - s), d, 2 * d, device=dev, generator=g)
        cov[s:s + X.shape[0]] = X @ X.transpose(1, 2) / (2 * d) + 0.25 * torch.eye(d, device=dev)
    consts = torch.zeros(5, d, d, dtype=torch.float64, device=dev)
    consts[0] = torch.eye(d, dtype=torch.float64) * 0.5
    consts[1] = torch.eye(d, dtype=torch.float64) * 2.0 + 0.01
    out = torch.zeros(T * n * 4, dtype=torch.float64, device=dev)
    dims = _lib.ame_dims(n, r, T, 0, T, 0)
    args = _lib.ame_cov_args(cov=cov.data_ptr(), consts=consts.data_ptr(), cov_terms=out.data_ptr())
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        for _ in range(3):
            _lib.check(L.ame_cov(ctypes.byref(dims), ctypes.byref(args), sp), "ame_cov")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            _lib.check(L.ame_cov(ctypes.byref(dims), ctypes.byref(args), sp), "ame_cov")
        e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    alg = 4.0 * n * T * d * d
    print(json.dumps({"ms": ms, "frac": alg / (ms * 1e-3) / 8e12, "finite": bool(torch.isfinite(out).all())}))


def main():
    args = sys.argv[1:]
    if args and args[0] == "--worker":
        n, T, r, reps = (int(x) for x in args[1:5])
        worker(n, T, r, reps)
        return
    shapes, rounds, reps = "4096,32,32;1024,128,16", 3, 20
    libs = []
    i = 0
    while i < len(args):
        if args[i] == "--shapes":
            shapes = args[i + 1]; i += 2
        elif args[i] == "--rounds":
            rounds = int(args[i + 1]); i += 2
        elif args[i] == "--reps":
            reps = int(args[i + 1]); i += 2
        else:
            libs.append(args[i]); i += 1
    res = {}
    for rnd in range(rounds):
        for shp in shapes.split(";"):
            n, T, r = (int(x) for x in shp.split(","))
            for lib in libs:
                env = dict(os.environ, AME_LIB_PATH=lib)
                out = subprocess.run([sys.executable, "-u", __file__, "--worker", str(n), str(T), str(r), str(reps)],
                                     env=env, capture_output=True, text=True, timeout=300)
                if out.returncode != 0:
                    print(out.stderr[-3000:])
                    sys.exit(1)
                v = json.loads(out.stdout.strip().splitlines()[-1])
                res.setdefault((shp, lib), []).append(v["ms"])
                print(f"round {rnd} n,T,r={shp} {os.path.basename(lib)}: {v['ms']:.4f} ms, "
                      f"HBM frac {v['frac']:.3f}, finite {v['finite']}", flush=True)
    for (shp, lib), v in res.items():
        print(f"{shp} {os.path.basename(lib)} median {sorted(v)[len(v) // 2]:.4f} ms {[round(x, 4) for x in v]}")


if __name__ == "__main__":
    main()
