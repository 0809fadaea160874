"""Diagnostic: per-phase cycle shares of one sweep step (in-kernel s_memtime stamps).

    python tools/sweep_stamps.py --build [--r=16]          # here: hipcc -DAME_STAMPS -> tools/_lib/libame_amd_stamps.so
    python tools/sweep_stamps.py [--n=1024 --T=128 --r=16 --variant=good --kind=20] # GPU box: v2 sweep, phase shares

Stamps are taken by thread 0 of the middle lane for 16 nodes in steady state.
The stamped build's run time is never quoted; only its SHARES are meaningful.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "python-temporal-ame-svi_amd")
BDIR = os.path.join(PKG, "ame_amd", "_build")      # objects (not shipped to the GPU box)
LIBDIR = os.path.join(ROOT, "tools", "_lib")         # variant libraries (shipped)
SO = os.path.join(LIBDIR, "libame_amd_stamps.so")
AME_STAMP_I0 = 256   # ame_sweep.hip
PHASES = ["phase 1: K-matvecs + z staging", "phase 2: wave0 Woodbury | waves1-3 GEMV+poll",
          "phase 3: K rank-4 update + cov write + AR", "loop (+ cov prefetch issue)"]



def _unsplit_sources():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "python-temporal-ame-svi_amd"))
    from ame_amd.build import UNSPLIT_SOURCES
    return UNSPLIT_SOURCES

def _opt(name, default=None):
    for a in sys.argv:
        if a.startswith(name + "="):
            return a.split("=", 1)[1]
    return default


def build(r=16):
    """--defs=A,B adds -DA -DB (ablation switches); --tag=X names the library."""
    os.makedirs(BDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    csrc = os.path.join(PKG, "ame_amd", "csrc")
    defs = [f"-D{d}" for d in (_opt("--defs") or "").split(",") if d]
    tag = _opt("--tag", "")
    so = SO.replace(".so", f"{tag}.so")
    objs = []
    for src in _unsplit_sources():
        o = os.path.join(BDIR, src.replace(".hip", f"_stamps{tag}.o"))
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                               "-DAME_STAMPS", f"-DAME_ONLY_R={r}", *defs, "-Wno-pass-failed",
                               "-c", os.path.join(csrc, src), "-o", o])
        objs.append(o)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", so, *objs])
    print("built", so)


def run():
    os.environ["AME_LIB_PATH"] = SO.replace(".so", f"{_opt('--tag', '')}.so")
    n, T, r = int(_opt("--n", 1024)), int(_opt("--T", 128)), int(_opt("--r", 16))
    sys.path.insert(0, PKG)
    import torch
    from ame_amd import TemporalAMEModel, TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI
    from ame_amd import _lib
    dev = torch.device("cuda", 0)
    m = TemporalAMEModel(n, T, r, seed=42)
    m.generate_data_fast(device=dev)
    variant = _opt("--variant", "good")
    # the stamps live in the v2 kernel: request a v2 kind explicitly (AUTO would
    # pick v3 at n=1024, r=16, whose stamp buffer this tool does not read)
    kind = int(_opt("--kind", _lib.AME_SWEEP_V2_AUTO))
    opts = {"sweep_kernel": kind}
    if variant == "naive":
        vi = TemporalAMENaiveMFVI(m, learning_rate=0.01, device=dev, engine_options=opts)
    else:
        vi = TemporalAMEStructuredMFVI(m, factorization=variant, learning_rate=0.01, device=dev,
                                       engine_options=opts)
    assert vi.engine.sweep_kind in (_lib.AME_SWEEP_V2_LDS, _lib.AME_SWEEP_V2_HBM,
                                    _lib.AME_SWEEP_V2_WORKERS, _lib.AME_SWEEP_V2_PIPE,
                                    _lib.AME_SWEEP_V2_W6), vi.engine.sweep_kind
    # one launch per sweep (the stamp buffers are per kernel, not per group)
    assert len(vi.engine.groups) == 1, vi.engine.groups
    vi.fit(max_iter=2, tolerance=0.0, verbose=False)
    torch.cuda.synchronize()
    L = _lib.lib()
    L.ame_debug_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    NPH = 32
    buf = (ctypes.c_ulonglong * (16 * NPH))()
    assert L.ame_debug_read_stamps(buf, 16 * NPH) == 0
    rows = [[buf[k * NPH + p] for p in range(NPH)] for k in range(16)]
    nph = len(PHASES)
    tot = [0.0] * nph
    step = []
    for k in range(15):
        r, nxt = rows[k], rows[k + 1]
        seq = r[:nph] + [nxt[0]]
        for p in range(nph):
            tot[p] += seq[p + 1] - seq[p]
        step.append(nxt[0] - r[0])
    T = sum(tot)
    print(f"mean step {sum(step) / len(step):.0f} cycles (s_memtime ticks)")
    for name, t in zip(PHASES, tot):
        print(f"  {name:48s} {t / 15:9.0f}  {100 * t / T:5.1f}%")
    sub = {4: "w0 matvec items done", 5: "w2 matvec items done", 6: "w3 matvec items done",
           7: "w0 z staged", 8: "w0 multidot-1 done", 9: "w0 mean published",
           10: "w0 multidot-2 done", 11: "w1 gemv done", 12: "w1 poll done",
           13: "w2 gemv done", 14: "w0 K update + cov write done", 15: "w0 gemv_reduce+AR done"}
    base = {4: 0, 5: 0, 6: 0, 7: 0, 8: 1, 9: 1, 10: 1, 11: 1, 12: 1, 13: 1, 14: 2, 15: 2}
    if any(rows[k][16] for k in range(15)):   # fine slots (kind 22)
        sub.update({16: "w0 cov park", 17: "w0 cov flush + prefetch issued", 18: "w0 W/Y item",
                    19: "w0 chunk", 20: "w2 loads issued", 21: "w2 W/Y item", 22: "w2 chunk",
                    23: "w2 right/old rows parked", 24: "w2 gather done", 25: "w2 ar_right",
                    26: "w1 gemv_reduce", 27: "w2 gemv_reduce", 28: "w0 gob summed"})
        base.update({16: 0, 17: 0, 18: 0, 19: 0, 20: 0, 21: 0, 22: 0, 23: 0, 24: 1, 25: 1,
                     26: 1, 27: 1, 28: 2})
    for ph in sorted(sub):
        d = sum(rows[k][ph] - rows[k][base[ph]] for k in range(15)) / 15
        print(f"    +{d:8.0f} after phase start: {sub[ph]}")
    if hasattr(L, "ame_debug_read_p2stamps"):   # phase 2 of waves 1-3 (kind 22)
        L.ame_debug_read_p2stamps.argtypes = [ctypes.c_void_p]
        pb = (ctypes.c_ulonglong * (16 * 16))()
        if L.ame_debug_read_p2stamps(pb) == 0 and pb[0]:
            names = {0: "w1 signalled", 2: "w2 signalled", 4: "w3 signalled", 6: "AR-left done (last wave)",
                     1: "w1 reduce+AR done", 3: "w2 reduce+AR done", 5: "w3 reduce+AR done",
                     8: "w1 AR-left start", 9: "w1 AR-left end", 10: "w2 AR-left start", 11: "w2 AR-left end",
                     12: "w3 AR-left start", 13: "w3 AR-left end"}
            for sl in sorted(names):
                d = sorted(pb[k * 16 + sl] - rows[k][1] for k in range(15))[7]
                print(f"    +{d:8d} after phase-2 start: {names[sl]}")
            d = sorted(pb[k * 16 + 7] - rows[k][0] for k in range(15))[7]
            print(f"    +{d:8d} after phase-1 start: w1 matvec items done")
    if hasattr(L, "ame_debug_read_wstamps"):   # GEMV worker 0 of the same slice (kind 22)
        L.ame_debug_read_wstamps.argtypes = [ctypes.c_void_p]
        wb = (ctypes.c_ulonglong * (16 * 8))()
        if L.ame_debug_read_wstamps(wb) == 0 and wb[0]:
            w = [[wb[k * 8 + p] for p in range(8)] for k in range(16)]
            per = [w[k + 1][0] - w[k][0] for k in range(15)]
            print(f"worker 0: mean node period {sum(per) / 15:.0f} cycles; phases (median over 16 nodes):")
            for p, nm in enumerate(["node m-4 seen", "z staged", "GEMV done", "partial stored"], 1):
                d = sorted(w[k][p] - w[k][p - 1] for k in range(16))[8]
                print(f"    {nm:16s} +{d:7d}")
            # when partial m (worker) was stored vs main's step m-1 start (node m-1 = I0+3+k)
            # (s_memtime counters of different XCDs are not comparable: the lead
            # uses the device-wide s_memrealtime recorded beside each stamp, 100 MHz)
            if hasattr(L, "ame_debug_read_rt"):
                L.ame_debug_read_rt.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
                mrt = (ctypes.c_ulonglong * (16 * 32))()
                wrt = (ctypes.c_ulonglong * (16 * 8))()
                if L.ame_debug_read_rt(mrt, wrt) == 0:
                    # main step i = I0 + k: phase-2 start (stamp 1) and gather(i+1) done
                    # (stamp 24); worker partial m = i + 1 stored: wrt[(i + 1 - I0 - 4) * 8 + 4]
                    lead, gwait = [], []
                    for k in range(3, 16):
                        wi = (k + 1 - 4) * 8 + 4
                        if mrt[k * 32 + 1] and wrt[wi]:
                            lead.append((mrt[k * 32 + 1] - wrt[wi]) * 10.0)        # ns
                            gwait.append((mrt[k * 32 + 24] - mrt[k * 32 + 1]) * 10.0)
                    if lead:
                        print(f"    main phase-2 start of step m-1 minus partial m stored (ns, >0: "
                              f"ready early): median {sorted(lead)[len(lead) // 2]:.0f}, "
                              f"min {min(lead):.0f}, max {max(lead):.0f}")
                        print(f"    main gather(m) done minus phase-2 start (ns): median "
                              f"{sorted(gwait)[len(gwait) // 2]:.0f}")
    if hasattr(L, "ame_debug_read_lag"):   # wavefront lag between consecutive slices
        L.ame_debug_read_lag.argtypes = [ctypes.c_void_p]
        lb = (ctypes.c_ulonglong * 512)()
        TL = min(vi.engine.groups[0][1], 64)   # (offset, size) of the one group
        if L.ame_debug_read_lag(lb) == 0 and lb[0]:
            s0 = [lb[8 * t] for t in range(TL)]
            s1 = [lb[8 * t + 1] for t in range(TL)]
            st = [lb[8 * t + 2] for t in range(TL)]
            per = sorted((s1[t] - s0[t]) * 10.0 / 64 for t in range(TL))      # ns per step
            lag = sorted((s0[t] - s0[t - 1]) * 10.0 for t in range(1, TL))    # ns
            p = per[len(per) // 2]
            print(f"wavefront: node period {p:.0f} ns (median over {TL} slices, steps "
                  f"{AME_STAMP_I0}..{AME_STAMP_I0 + 64}); slice-to-slice lag at step {AME_STAMP_I0}: "
                  f"median {lag[len(lag) // 2]:.0f} ns = {lag[len(lag) // 2] / p:.2f} steps, "
                  f"min {lag[0] / p:.2f}, max {lag[-1] / p:.2f}; last slice - first slice "
                  f"{(s0[-1] - s0[0]) * 10.0 / p:.1f} steps over {TL - 1} hops")
            t0 = min(st)
            print("  per slice (steps of that period, from the earliest step-0 start): step 0 at / "
                  f"step {AME_STAMP_I0} at")
            eb = None
            if hasattr(L, "ame_debug_read_entry"):
                L.ame_debug_read_entry.argtypes = [ctypes.c_void_p]
                eb = (ctypes.c_ulonglong * 1024)()
                if L.ame_debug_read_entry(eb) != 0 or not eb[0]:
                    eb = None
            NG = {_lib.AME_SWEEP_V2_WORKERS: 7, _lib.AME_SWEEP_V2_W6: 6}.get(vi.engine.sweep_kind, 0)
            if eb is not None:
                nb = TL * (1 + NG)
                e0 = min(eb[2 * b] for b in range(nb))
                print("  workgroup entry (kernel start), steps after the first workgroup's entry; "
                      "main workgroup / last of its workers; then step 0 / step 256 from the earliest step 0")
            for t in range(TL):
                extra = ""
                if eb is not None:
                    me = (eb[2 * t] - e0) * 10.0 / p
                    ws = [TL + NG * t + w for w in range(NG)]
                    we = max((eb[2 * b] - e0) * 10.0 / p for b in ws) if ws else 0.0
                    hid = eb[2 * t + 1]
                    mk = [(lb[8 * t + j] - e0) * 10.0 / p if lb[8 * t + j] else float("nan")
                          for j in (6, 5, 3, 7, 4, 2)]
                    extra = (f"   entry {me:6.1f} / {we:6.1f}  w0 loop {mk[0]:7.1f}  w0 part0 {mk[1]:7.1f}"
                             f"  left0|sums {mk[2]:7.1f}  P0inv {mk[3]:7.1f}  gather0 {mk[4]:7.1f}"
                             f"  step0 {mk[5]:7.1f}"
                             f"  xcc {hid >> 32}")
                print(f"    slice {t:3d}: {(st[t] - t0) * 10.0 / p:8.1f}  {(s0[t] - t0) * 10.0 / p:8.1f}{extra}")
            if eb is not None:
                late = sorted(((eb[2 * b] - e0) * 10.0 / p, b) for b in range(nb))[-6:]
                print("  latest workgroup entries (steps, blockIdx):", [(round(x, 1), b) for x, b in late])


if __name__ == "__main__":
    build(int(_opt("--r", 16))) if "--build" in sys.argv else run()
