"""Run-to-run determinism of the sweep at config 3's shape (n=1024, T=128, r=16):
fits from the same seed must give bit-equal means, single-process and split
over two ranks on one GPU (peer-buffer halo).  Prints the first
(iteration, node, slice) that differs.   GPU box:  python tools/determinism.py [reps]

Other cases through the environment: DET_SHAPE=n,T,r  DET_VARIANT=good|bad|naive
DET_WORLD=ranks  DET_LR  DET_ITERS  DET_DEPTH (queue depth)  DET_SEEDS=model,data
(e.g. the tests/test_gpu_distributed.py case 4 ranks, 64,16,3, bad, 0.8, 8, 3, 21,4).
"""
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-temporal-ame-svi_amd"))
ITERS = int(os.environ.get("DET_ITERS", "3"))
SHAPE = tuple(int(x) for x in os.environ.get("DET_SHAPE", "1024,128,16").split(","))
VARIANT = os.environ.get("DET_VARIANT", "good")
WORLD = int(os.environ.get("DET_WORLD", "2"))
LR = float(os.environ.get("DET_LR", "0.01"))
DEPTH = os.environ.get("DET_DEPTH")
SEEDS = tuple(int(x) for x in os.environ.get("DET_SEEDS", "42,-1").split(","))


def run(distributed):
    import torch
    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    dev = torch.device("cuda", 0)
    m = TemporalAMEModel(*SHAPE, seed=SEEDS[0])
    if SEEDS[1] >= 0:
        m.generate_data_fast(seed=SEEDS[1])
    else:
        m.generate_data_fast(device=dev)
    opts = {} if DEPTH is None else {"spec_depth": int(DEPTH)}
    if VARIANT == "naive":
        vi = TemporalAMENaiveMFVI(m, learning_rate=LR, device=dev, distributed=distributed,
                                  engine_options=opts)
    else:
        vi = TemporalAMEStructuredMFVI(m, factorization=VARIANT, learning_rate=LR, device=dev,
                                       distributed=distributed, engine_options=opts)
    out = []
    if os.environ.get("DET_PIPELINED", "1") == "1":   # one fit: pipelined sweeps
        vi.fit(max_iter=ITERS, tolerance=0.0, verbose=False)
        out.append(vi.X_mean.numpy().copy())
        return out
    for _ in range(ITERS):
        vi.fit(max_iter=1, tolerance=0.0, verbose=False)
        out.append(vi.X_mean.numpy().copy())
    return out


def worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = run(True)
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def run_dist():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = q.get(timeout=150)
    for p in procs:
        p.join(timeout=30)
    return out


def compare(tag, a, b):
    ok = True
    for it, (ma, mb) in enumerate(zip(a, b)):
        d = np.argwhere(ma != mb)
        if len(d):
            ok = False
            print(f"  {tag} iter {it}: {len(d)} mean diffs, max {np.abs(ma - mb).max():.3e}, "
                  f"first (node, t, k) {d[:6].tolist()}, slices {sorted(set(d[:, 1].tolist()))[:12]}")
    return ok


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ref = run(None)
    bad = 0
    for r in range(reps):
        ok = compare(f"single rep {r}", ref, run(None))
        ok &= compare(f"{WORLD}-rank rep {r}", ref, run_dist())
        print(f"rep {r}: {'equal' if ok else 'DIFFERENT'}", flush=True)
        bad += not ok
    print("DETERMINISTIC" if bad == 0 else f"NONDETERMINISTIC in {bad}/{reps} reps")


if __name__ == "__main__":
    main()
