"""Device engine: HBM-resident VI state + the per-iteration kernel sequence.

One engine per process / GPU.  It owns, for the local time slices
[t_begin, t_begin + T_local):

    Yt        [T_local][n][ny][2] fp32  observed network, time-major, rows padded to
                                        even length (ame_pack_y)
    xs[k]     [T_local][n][d]    fp32   means: ring of spec_depth + 1 states
    covs[k]   [T_local][n][d][d] fp32   covariances: same ring (x_a / cov = current)
    hand      [T_local][n][d]    u64    lane-to-lane {epoch,value} granules
    cov_terms [T_local][n][4]    fp64   per-(node,time) covariance ELBO terms

and runs, per fit() iteration (reference base.py:170-181):

    ame_sweep   (means + covariances)       structured_mf.py:211-326
    ame_cov     (covariance ELBO terms)     structured_mf.py:142-144, 166, 193, 202-209
    ame_elbo    (pair + node sums)          structured_mf.py:115-200, temporal_ame.py:255-291

The host then assembles ELBO and MSE from 8 fp64 sums (+ the analytic
constants) exactly as the reference's formulas define them.

A sweep reads the current state and writes the spare buffers, which become
current when the sweep is committed.  While fit() has another iteration to
go, the next sweep does not depend on this iteration's ELBO, so it is started
on a high-priority stream of its own before this iteration's ELBO kernels,
which then run beside it on the main stream (they read only the current
state); the next update_step merely commits it.  When fit() stops instead
(convergence or max_iter) the started sweep is dropped: it never touched the
current state.  On one GPU, when both sweeps' workgroups fit on the chip,
the next sweep is queued while the previous one still runs (pipelined): each
of its slices waits on the device for the previous sweep to finish slices t
and t+1, so consecutive sweeps overlap and the wavefront fill is paid once per
fit() instead of once per iteration.  Results are bit-identical to running
the kernels in order (tests/test_gpu_parity.py::test_speculative_sweep_is_exact).
"""
from __future__ import annotations

import collections
import ctypes
import math
import time
from dataclasses import dataclass, fields
from typing import Optional

import torch

from . import _lib

LOG2PI = math.log(2.0 * math.pi)
VARIANTS = {"good": _lib.AME_GOOD, "bad": _lib.AME_BAD, "naive": _lib.AME_NAIVE}


@dataclass
class Shard:
    """Contiguous block of time slices held by this rank."""
    t_begin: int
    T_local: int
    T_total: int
    rank: int = 0
    world: int = 1


# CU-masked streams (EngineOptions.elbo_cus), per (device, first CU, CUs, slot)
_CU_STREAMS = {}


@dataclass
class EngineOptions:
    """Execution choices of one engine.  Nothing is read from the environment:
    the defaults are the production path, tests and A/B runs pass these
    explicitly (``engine_options=`` of the VI classes).

    sweep_kernel  request code of include/ame_amd.h (``_lib.AME_SWEEP_*``):
                  AUTO picks v3 when the shape fits it, else v2 (with GEMV
                  workers when they are co-resident)
    pipeline      queue the next sweep while this one runs (kernels that order
                  themselves slice by slice on the device)
    speculate     start the next sweep before this iteration's ELBO is read
    spec_depth    sweeps kept started ahead of the committed state when
                  pipelined; None derives it from the global slice count
                  (:func:`derive_spec_depth`)
    slice_group   at most this many local slices per launch (0: as many as fit)
    pairs_kernel  ELBO pair kernel (``_lib.AME_PAIRS_*``; 0 = default)
    elbo_cus      > 0: run the ELBO kernels on their own CU-masked stream over
                  compute units [0, elbo_cus) and the sweep streams over the
                  rest (ame_stream_create_cu_range), so iteration k's ELBO runs
                  beside sweep k+1 instead of queueing behind its workgroups.
                  Needs a non-pipelined GEMV-worker kind (sweep_kernel 22 or 24)
                  whose launch fits the remaining CUs (kind 24 at config 5's
                  rank shape: 32 slices x 7 workgroups = 224 CUs, elbo_cus 32)
    elbo_first    queue this iteration's ELBO kernels before the speculative
                  next sweep and order that sweep after them (default: after
                  it).  Same results; measured at config 5's rank shape (kind
                  22) no faster: 32.8-35.5 vs 33.0-34.0 ms per iteration
                  (profiles/r05_c5_elbo_first_ab.txt), so off
    """
    sweep_kernel: int = 0
    pipeline: bool = True
    speculate: bool = True
    spec_depth: Optional[int] = None
    slice_group: int = 0
    pairs_kernel: int = 0
    elbo_cus: int = 0
    elbo_first: bool = False

    @classmethod
    def coerce(cls, opts) -> "EngineOptions":
        if opts is None:
            return cls()
        if isinstance(opts, cls):
            return opts
        names = {f.name for f in fields(cls)}
        bad = set(opts) - names
        if bad:
            raise ValueError(f"unknown engine option(s) {sorted(bad)}; known: {sorted(names)}")
        return cls(**opts)


# Queue-depth model.  In the pipelined steady state with period
# P (about one slice's chain of n node steps) the host reads iteration k's ELBO
# once sweep k has finished on the LAST slice of the LAST rank, i.e. after the
# wavefront's fill over all T_total slices plus one chain plus the ELBO kernels
# and the all_reduce; by then sweep k + 1 + depth must already be queued:
#     (1 + depth) P >= fill + C + delta,   fill = F (T_total - 1) steps.
# F = node steps of lag per slice: 2.94 measured in round 4 (lane start offset
# 890 us over 127 slices at 2.38 us per step, profiles/r04_v3_stamps_head.txt;
# 2.6 in round 1), rounded up to 3.0 -- a deeper queue only costs a state slot;
# delta ~ 128 steps (0.33 ms).
FILL_STEPS_PER_SLICE = 3.0
ELBO_READ_STEPS = 128
MAX_SPEC_DEPTH = 8


def derive_spec_depth(n: int, T_total: int) -> int:
    """Smallest queue depth the model above needs, at least 2 (measured best on
    one GPU), at most MAX_SPEC_DEPTH."""
    need = math.ceil((FILL_STEPS_PER_SLICE * (T_total - 1) + ELBO_READ_STEPS) / max(1, n))
    return max(2, min(MAX_SPEC_DEPTH, need))


# Sweep epochs are unique within the process: every engine starts above the
# highest epoch any earlier engine launched.  A buffer the caching allocator
# recycles from an older engine (done flags, hand-off granules) then only
# holds epochs BELOW every epoch this engine waits for, so a stale word makes
# a waiter wait instead of passing; the device additionally flags any word
# ABOVE the epoch window (AME_STATUS_STALE_EPOCH, include/ame_amd.h).
_EPOCH_HIGH = 0


def _epoch_base() -> int:
    return _EPOCH_HIGH


def _note_epoch(e: int) -> None:
    global _EPOCH_HIGH
    _EPOCH_HIGH = max(_EPOCH_HIGH, int(e))


_STATUS_TEXT = (
    (_lib.AME_STATUS_SPIN_TIMEOUT, "a hand-off between slices timed out (workgroups not co-resident?)"),
    (_lib.AME_STATUS_HALO_TIMEOUT, "a hand-off from a neighbouring rank timed out"),
    (_lib.AME_STATUS_LDS_TIMEOUT, "an intra-workgroup hand-off timed out (internal error)"),
    (_lib.AME_STATUS_STALE_EPOCH, "a hand-off word carried an epoch outside the protocol's "
                                  "window (stale buffer or an unordered write): results of "
                                  "this sweep are not trusted"),
)


def status_text(st: int) -> str:
    parts = [txt for bit, txt in _STATUS_TEXT if st & bit]
    return "; ".join(parts) if parts else "unknown"


def status_report(words) -> str:
    """Text of a status block (include/ame_amd.h, AME_STATUS_WORDS uint32):
    the bits, then the record of the FIRST failing wait (site, slice, node,
    word seen vs expected, time waited, sweep epoch) and how many later waits
    gave up quietly because of it."""
    w = [int(x) & 0xFFFFFFFF for x in words]
    w += [0] * (_lib.AME_STATUS_WORDS - len(w))
    msg = f"device status {w[0]:#x}: {status_text(w[0])}"
    if w[1]:
        node = "prologue" if w[4] == 0xFFFFFFFF else f"node {w[4]}"
        site = _lib.AME_WAIT_SITES.get(w[2], f"site {w[2]}")
        msg += (f"; first failure: {site}, slice {w[3]}, {node}, saw {w[5]} expected {w[6]}, "
                f"after {w[7] / 1e3:.1f} ms, sweep epoch {w[8]}")
    if w[10]:
        msg += f"; {w[10]} later wait(s) gave up quietly"
    return msg


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _blockdiag(Sigma, Psi):
    d = 2 + Psi.shape[0]
    S = torch.zeros(d, d, dtype=torch.float64)
    S[:2, :2] = Sigma.double()
    S[2:, 2:] = Psi.double()
    return S


def _sym(a):
    return 0.5 * (a + a.T)


class Constants:
    """fp64 model constants, built from the fp32 model attributes the reference reads."""

    def __init__(self, model):
        d = model.d
        self.R = model.R.detach().double().cpu()
        self.R_inv = model.R_inv.detach().double().cpu()
        S0 = _blockdiag(model.Sigma.detach().cpu(), model.Psi.detach().cpu())
        Q = model.Q.detach().double().cpu()
        Phi = model.Phi.detach().double().cpu()
        self.S0inv = _sym(torch.linalg.inv(S0))
        self.Qinv = _sym(torch.linalg.inv(Q))
        self.PtQiP = _sym(Phi.T @ self.Qinv @ Phi)
        self.QiPhi = self.Qinv @ Phi
        self.PhiTQi = Phi.T @ self.Qinv
        self.Phi = Phi
        self.logdetR = float(torch.logdet(self.R))
        self.trRinv = float(torch.trace(self.R_inv))
        self.logdetS0 = float(torch.logdet(S0))
        self.logdetQ = float(torch.logdet(Q))
        self.stack = torch.stack([self.S0inv, self.Qinv, self.PtQiP, self.QiPhi,
                                  self.PhiTQi]).contiguous()
        self.d = d

    def rinv4(self):
        r = self.R_inv.flatten().tolist()
        return (ctypes.c_double * 4)(*r)


def assemble(out, n, T, d, variant, C: Constants):
    """ELBO pieces and MSE from the 8 device sums (see include/ame_amd.h).

    Formulas: structured_mf.py:124-209 / naive_mf.py:114-191 and
    temporal_ame.py:290 with the pairwise correction collapsed as
    sum_{i<j}(tr_i + tr_j) = (n-1) sum_i tr_i.
    """
    npairs = T * n * (n - 1) / 2.0
    corr = 0.0 if variant == "naive" else 0.1 * C.trRinv / d * (n - 1) * out[1]
    loglik = -0.5 * (npairs * (C.logdetR + 2 * LOG2PI) + out[0] + corr)
    prior0 = -0.5 * (n * (C.logdetS0 + d * LOG2PI) + out[2] + out[3])
    trans = -0.5 * (n * (T - 1) * (C.logdetQ + d * LOG2PI) + out[4] + out[5])
    ent = 0.5 * (n * T * d * (1 + LOG2PI) + out[6])
    recon = out[7] / (n * (n - 1) * T)
    return {"loglik": loglik, "prior0": prior0, "trans": trans, "entropy": ent,
            "elbo": loglik + prior0 + trans + ent, "recon": recon}


def slice_groups(T_local: int, max_slices: int, force: int = 0):
    """Consecutive groups [(offset, size)] of the local slices that each fit on
    the chip at once (a sweep's slices spin on each other, so all slices of one
    launch must be co-resident).  The groups of one sweep run one after another
    on one stream; group g+1's first slice takes slice (g's last)'s new means
    from the hand-off granules group g left behind, so the Gauss-Seidel order
    is the same as one launch over all slices (reference: the t loop of
    structured_mf.py:240 has no limit on T)."""
    cap = max_slices if force <= 0 else min(force, max_slices)
    if cap < 1:
        raise RuntimeError("ame_amd: no sweep workgroup fits on this device")
    k = -(-T_local // cap)
    base, extra = divmod(T_local, k)
    out, off = [], 0
    for g in range(k):
        sz = base + (1 if g < extra else 0)
        out.append((off, sz))
        off += sz
    return out


class DeviceEngine:
    """HBM-resident state of one VI run on one GPU (one time shard)."""

    def __init__(self, model, variant: str, lr: float, X_mean: torch.Tensor,
                 X_cov: torch.Tensor, device=None, shard: Optional[Shard] = None,
                 halo=None, options: Optional[EngineOptions] = None):
        if not torch.cuda.is_available():
            raise RuntimeError("ame_amd: no GPU visible; the HIP path has no CPU fallback")
        self.L = _lib.lib()
        if variant not in VARIANTS:
            raise ValueError(f"Unknown factorization '{variant}'")
        self.variant = variant
        self.vcode = VARIANTS[variant]
        self.n, self.T, self.d, self.r = int(model.n), int(model.T), int(model.d), int(model.r)
        if self.r not in _lib.supported_r():
            raise RuntimeError(f"ame_amd: latent_dim={self.r} not compiled "
                               f"(supported {_lib.supported_r()})")
        self.dev = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.shard = shard or Shard(0, self.T, self.T)
        self.halo = halo
        self.options = opt = EngineOptions.coerce(options)
        self.lr = float(lr)
        self.C = Constants(model)
        sh = self.shard
        self.dims = _lib.ame_dims(self.n, self.r, sh.T_local, sh.t_begin, sh.T_total, self.vcode)
        dev = self.dev
        with torch.cuda.device(dev):
            self.stream = torch.cuda.current_stream(dev)
            self.consts = self.C.stack.to(dev)
            self.phi = self.C.Phi.contiguous().to(dev)
            self._pack_y(model.Y)
            t0, t1 = sh.t_begin, sh.t_begin + sh.T_local
            x0 = X_mean[:, t0:t1].detach().float().permute(1, 0, 2).contiguous().to(dev)
            c0 = X_cov[:, t0:t1].detach().float().permute(1, 0, 2, 3).contiguous().to(dev)
            self.xs, self.covs = [x0], [c0]
            self._cur = 0
            n, d, TL = self.n, self.d, sh.T_local
            self.hand = torch.zeros(TL * n * d, dtype=torch.int64, device=dev)
            self.cov_terms = torch.zeros(TL * n * 4, dtype=torch.float64, device=dev)
            ws = int(self.L.ame_elbo_work_size(ctypes.byref(self.dims)))
            if ws < 0:
                _lib.check(-1, "ame_elbo_work_size")
            self.work = torch.empty(ws, dtype=torch.float64, device=dev)
            self.out = torch.zeros(8, dtype=torch.float64, device=dev)
            self.status = torch.zeros(_lib.AME_STATUS_WORDS, dtype=torch.int32, device=dev)
        self.last_status = None   # the status block of the last failure _check_status raised
        self.epoch = _epoch_base()
        if self.halo is not None:   # every rank's sweep k carries the same epoch
            self.epoch = self.halo.agree_max(self, self.epoch)
        self.max_slices = int(self.L.ame_sweep_max_slices(self.n, self.r, opt.sweep_kernel))
        if self.max_slices < 1:
            raise RuntimeError(f"ame_amd: no sweep kernel fits n={self.n}, r={self.r} "
                               f"(request {opt.sweep_kernel})")
        self._cu_split = None
        if opt.elbo_cus:
            # ELBO beside the sweep: the sweep's launch must fit the CUs left to it
            # (workgroups per slice from the library, one CU each)
            per_slice = None
            if opt.sweep_kernel in (_lib.AME_SWEEP_V2_WORKERS, _lib.AME_SWEEP_V2_W6):
                per_slice = int(self.L.ame_sweep_slice_workgroups(opt.sweep_kernel))
            cus = int(torch.cuda.get_device_properties(self.dev).multi_processor_count)
            if per_slice is None or per_slice < 1 or not 0 < int(opt.elbo_cus) < cus:
                raise ValueError("elbo_cus needs sweep_kernel 22 or 24 and 0 < elbo_cus < "
                                 f"{cus} CUs (got {opt.elbo_cus}, kernel {opt.sweep_kernel})")
            self.max_slices = min(self.max_slices, (cus - int(opt.elbo_cus)) // per_slice)
            if self.max_slices < 1:
                raise ValueError(f"elbo_cus={opt.elbo_cus} leaves no room for a slice")
            self._cu_split = (int(opt.elbo_cus), cus)
        req = opt.sweep_kernel
        if req in (_lib.AME_SWEEP_AUTO, _lib.AME_SWEEP_V2_AUTO) and (
                req == _lib.AME_SWEEP_V2_AUTO
                or int(self.L.ame_sweep_max_slices(self.n, self.r, _lib.AME_SWEEP_V3)) < 1):
            # beyond v3's reach the GEMV-worker sweep (kind 22) in slice groups of
            # what co-resides beats ONE launch of the single-workgroup sweep over
            # all slices: config 5 at T = 256 on one GPU, 8 groups of 32 vs kind 21,
            # 285-302 vs 580 ms per iteration; the pipelined kind 23 in overlapping
            # groups measured the same, 274-291 ms, and loses at
            # T_local = 32, so kind 22 stays the choice.  AUTO picks kind 22
            # whenever T_local fits one launch
            w = int(self.L.ame_sweep_max_slices(self.n, self.r, _lib.AME_SWEEP_V2_WORKERS))
            if 1 <= w < min(sh.T_local, self.max_slices):
                gd = _lib.ame_dims(self.n, self.r, w, sh.t_begin, sh.T_total, self.vcode)
                if int(self.L.ame_sweep_kind(ctypes.byref(gd), req)) == _lib.AME_SWEEP_V2_WORKERS:
                    self.max_slices = w
        # Ranks of one time-sharded run that share this GPU share its CUs, and a
        # spinning launch of one rank can wait on a slice of another (halo, back
        # channel): all of them must be co-resident at once, so each rank
        # budgets for 1/k of the chip (co-residency rule)
        self.device_sharers = self.halo.device_sharers(self) if self.halo is not None else 1
        if self.device_sharers > 1:
            self.max_slices //= self.device_sharers
            if self.max_slices < 1:
                raise RuntimeError(f"ame_amd: {self.device_sharers} ranks share this GPU and one "
                                   f"sweep slice (n={self.n}, r={self.r}) does not fit 1/"
                                   f"{self.device_sharers} of it")
        # Pipelined layout: a kernel that orders itself slice by slice on the
        # device (done flags) runs with TWO launches co-resident -- consecutive
        # sweeps, and consecutive slice groups of one sweep -- so each launch gets
        # at most half of what co-resides; the launches alternate over two
        # streams
        pipe_cap = 0
        if opt.pipeline and self.max_slices >= 2:
            half = self.max_slices // 2
            pd = _lib.ame_dims(self.n, self.r, max(1, min(sh.T_local, half)), sh.t_begin,
                               sh.T_total, self.vcode)
            pk = int(self.L.ame_sweep_kind(ctypes.byref(pd), req))
            if pk >= 0 and bool(self.L.ame_sweep_orders_slices(self.n, self.r, pk)):
                pipe_cap = half
        self.groups = slice_groups(sh.T_local, pipe_cap or self.max_slices, opt.slice_group)
        # the kernel of each group size is resolved ONCE here and passed with
        # every launch (ame_sweep rejects a launch whose buffers were sized for
        # another kind); groups that run one after another share the scratch,
        # pipelined launches alternate between two halves of it
        self.group_kinds = {}
        sws = 1
        for size in sorted({sz for _, sz in self.groups}):
            gd = _lib.ame_dims(self.n, self.r, size, sh.t_begin, sh.T_total, self.vcode)
            k = int(self.L.ame_sweep_kind(ctypes.byref(gd), req))
            if k < 0:
                _lib.check(-1, "ame_sweep_kind")
            w = int(self.L.ame_sweep_work_size(ctypes.byref(gd), k))
            if w < 0:
                _lib.check(-1, "ame_sweep_work_size")
            self.group_kinds[size] = k
            sws = max(sws, w)
        self.sweep_kind = self.group_kinds[self.groups[0][1]]
        self._out_host = None
        self._out_valid = False
        self.timing = False       # record HIP events around each kernel launch
        self.events = []          # (name, start, end) while timing
        self.speculation = bool(opt.speculate)
        self._specs = collections.deque()   # (done events, ring slot) of sweeps started ahead
        # consecutive sweeps (or, pipelined, consecutive launches) alternate
        # between two high-priority streams
        self.elbo_stream = None
        if self._cu_split is None:
            self.sweep_streams = [torch.cuda.Stream(device=self.dev, priority=-1) for _ in range(2)]
        else:
            ec, cus = self._cu_split
            self.elbo_stream = self._cu_stream(0, ec)
            self.sweep_streams = [self._cu_stream(ec, cus - ec, slot) for slot in range(2)]
        self._launch_ctr = 0
        self.done = torch.zeros(max(sh.T_local, 1), dtype=torch.int32, device=self.dev)
        kinds = set(self.group_kinds.values())
        # slice workgroups of this kind the whole chip holds at once
        self.resident_slots = int(self.L.ame_sweep_max_slices(self.n, self.r, self.sweep_kind))
        self.pipelined = (len(kinds) == 1 and pipe_cap > 0
                          and bool(self.L.ame_sweep_orders_slices(self.n, self.r, self.sweep_kind))
                          and 2 * max(sz for _, sz in self.groups) * self.device_sharers
                          <= self.resident_slots
                          and bool(opt.pipeline))
        if self.halo is not None:   # every rank must take the same path
            self.pipelined = self.halo.agree(self, self.pipelined)
        # launches of this process that may spin at once (pipelined: one per
        # sweep stream); the co-residency rule is
        #     device_sharers * coresident_launches * largest group <= resident_slots
        self.coresident_launches = 2 if self.pipelined else 1
        # How many sweeps may run ahead of the committed state.  Pipelined sweeps
        # overlap slice by slice, so a deeper queue keeps the wavefront full when
        # its fill over all T slices (all ranks) exceeds one iteration: the host
        # reads iteration k's ELBO only after sweep k has finished everywhere, and
        # sweep k+depth must already be queued by then.
        if opt.spec_depth is None:
            self.spec_depth = derive_spec_depth(self.n, sh.T_total) if self.pipelined else 1
        else:
            self.spec_depth = int(opt.spec_depth)
        if self.spec_depth < 1:
            raise ValueError("spec_depth must be >= 1")
        if not self.pipelined:
            # A sweep that does not order itself slice by slice on the device must
            # not start before the sweep that writes its input slot has finished;
            # with more than one queued that is a serial chain anyway, so the
            # queue is one deep (_launch_sweep also orders after the last one).
            self.spec_depth = 1
        # ELBO before the speculative sweep (EngineOptions.elbo_first)
        self.elbo_first = bool(opt.elbo_first)
        if self.halo is not None:   # the collectives of sums() keep one order on every rank
            self.elbo_first = self.halo.agree(self, self.elbo_first)
        # scratch per launch; pipelined, two launches run at once: two halves
        self._work_half = sws
        with torch.cuda.device(dev):
            self.sweep_work = torch.empty(sws * (2 if self.pipelined else 1), dtype=torch.float64,
                                          device=dev)
            while len(self.xs) < self.spec_depth + 1:
                self.xs.append(torch.empty_like(self.xs[0]))
                self.covs.append(torch.empty_like(self.covs[0]))
        self._host_ready = None
        # test hook only (tests/test_gpu_stale_epoch.py): False lets a pipelined
        # launch skip the wait for host-issued writes, to show the device's
        # epoch-window check catching the resulting stale flags
        self._order_after_host_writes = True
        # test hook only (tests/test_gpu_skew.py): seconds this rank sleeps before
        # its first sweep launch, after that sweep's collectives -- a rank that
        # arrives late, as host jitter or a slow first collective makes it
        self._first_launch_delay_s = 0.0
        self._mark_host_writes()

    def _cu_stream(self, first, num, slot=0):
        """A stream over compute units [first, first + num) (C-ABI, HIP CU mask),
        shared by every engine of the process and never destroyed: the caching
        allocator keeps events on the streams its blocks were used on
        (record_stream), so a stream must outlive every tensor an engine drops."""
        key = (self.dev.index, int(first), int(num), int(slot))
        st = _CU_STREAMS.get(key)
        if st is None:
            p = ctypes.c_void_p()
            with torch.cuda.device(self.dev):
                _lib.check(self.L.ame_stream_create_cu_range(int(first), int(num), ctypes.byref(p)),
                           "ame_stream_create_cu_range")
            st = _CU_STREAMS[key] = torch.cuda.ExternalStream(p.value, device=self.dev)
        return st

    def _elbo_stream_begin(self):
        """The stream the ELBO kernels run on: the main stream, or (elbo_cus) the
        CU-masked ELBO stream ordered after everything queued on the main one."""
        if self.elbo_stream is None:
            return self.stream
        ev = torch.cuda.Event()
        ev.record(self.stream)
        self.elbo_stream.wait_event(ev)
        return self.elbo_stream

    def _elbo_stream_end(self, st):
        if st is not self.stream:   # later main-stream work (reading out) waits for it
            ev = torch.cuda.Event()
            ev.record(st)
            self.stream.wait_event(ev)

    def _mark_host_writes(self):
        """Record the main-stream position after host-issued writes to the state
        or the sweep's flags (uploads, zero fills, set_means / set_covs).  A
        pipelined launch orders itself on the device against the previous sweep
        only; this event orders it after these writes as well (its stream has no
        other tie to the main stream)."""
        ev = torch.cuda.Event()
        ev.record(self.stream)
        self._host_ready = ev

    # current state (ring slot _cur)
    @property
    def x_a(self) -> torch.Tensor:
        return self.xs[self._cur]

    @property
    def cov(self) -> torch.Tensor:
        return self.covs[self._cur]

    # ------------------------------------------------------------------
    def _sp(self):
        return ctypes.c_void_p(self.stream.cuda_stream)

    def _tic(self, name, stream=None):
        if not self.timing:
            return None
        s = self.stream if stream is None else stream
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        return (name, e, s)

    def _toc(self, tok, stream=None):
        if tok is None:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record(tok[2] if stream is None else stream)
        self.events.append((tok[0], tok[1], e))

    def kernel_ms(self):
        """Average device ms per launch of each timed kernel (synchronises)."""
        torch.cuda.synchronize(self.dev)
        acc = {}
        for name, a, b in self.events:
            acc.setdefault(name, []).append(a.elapsed_time(b))
        return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}

    def _pack_y(self, Y):
        if Y is None:
            raise ValueError("No data generated yet. Call generate_data() first.")
        sh = self.shard
        src = Y.detach()
        if src.dtype != torch.float32:
            src = src.float()
        src = src.to(self.dev).contiguous()
        ysz = int(self.L.ame_pack_y_size(ctypes.byref(self.dims)))
        if ysz < 0:
            _lib.check(-1, "ame_pack_y_size")
        self.ny = ysz // (2 * sh.T_local * self.n)   # row stride: n rounded up to even
        self.Yt = torch.empty(sh.T_local, self.n, self.ny, 2, dtype=torch.float32, device=self.dev)
        mm = torch.zeros(1, dtype=torch.int64, device=self.dev)
        rc = self.L.ame_pack_y(_ptr(src), _ptr(self.Yt), ctypes.byref(self.dims), _ptr(mm),
                               self._sp())
        _lib.check(rc, "ame_pack_y")
        self.swap_consistent = int(mm.item()) == 0
        del src

    # ------------------------------------------------------------------
    def _launch_sweep(self, spec=False):
        """Enqueue one sweep from the newest state (the last queued sweep's
        output, or the current state) into the next ring slot; returns
        (done-events, slot).
        A speculative sweep in pipelined mode is queued while the previous sweep
        (epoch - 1) still runs and orders itself slice by slice on the device;
        any other sweep is ordered after everything queued on the main stream.
        Pipelined engines alternate their launches -- sweeps and slice groups --
        over the two sweep streams, so launch j + 1 runs beside launch j and
        launch j + 2 queues behind launch j (at most two co-resident); otherwise
        a sweep's groups run in order on one stream."""
        src = self._specs[-1][1] if self._specs else self._cur
        dst = (src + 1) % len(self.xs)
        self.epoch += 1
        _note_epoch(self.epoch)
        pipe = spec and self.pipelined and self.speculation
        halo_in = halo_out = next_old = back_in = back_out = None
        if self.halo is not None:
            # a pipelined launch takes next_old from the back channel instead of a
            # collective that would wait for the running sweep
            next_old, halo_in, halo_out = self.halo.before_sweep(
                self, gather=not pipe, first=self.xs[src][0])
            back_in, back_out = self.halo.back_channels(self)
        if self._first_launch_delay_s:
            time.sleep(self._first_launch_delay_s)
            self._first_launch_delay_s = 0.0
        wait = self.epoch - 1 if pipe else 0
        ready = None
        if not pipe:
            ready = torch.cuda.Event()
            ready.record(self.stream)
        prev = self._specs[-1][0] if self._specs else []
        used = []

        def order(stream):   # first launch of this sweep on `stream`
            if stream in used:
                return
            used.append(stream)
            if pipe:
                if self._order_after_host_writes:
                    stream.wait_event(self._host_ready)
            else:
                stream.wait_event(ready)
                for ev in prev:   # its input slot is the output of the last queued sweep
                    stream.wait_event(ev)

        tok = None
        n, d, sh = self.n, self.d, self.shard
        last = len(self.groups) - 1
        stream = None
        for g, (off, size) in enumerate(self.groups):
            if self.pipelined:
                par = self._launch_ctr & 1
                self._launch_ctr += 1
            else:
                par = 0
            stream = self.sweep_streams[par if self.pipelined else (self.epoch & 1)]
            order(stream)
            if tok is None:
                tok = self._tic("sweep", stream)

            def at(t, slices, per_slice, esize):   # pointer to local slice `slices` of t
                return ctypes.c_void_p(t.data_ptr() + slices * per_slice * esize)
            nd, ndd, nn2 = n * d, n * d * d, n * self.ny * 2
            g_halo_in = halo_in if g == 0 else at(self.hand, off - 1, nd, 8)
            g_halo_out = halo_out if g == last else None
            g_next_old = next_old if g == last else at(self.xs[src], off + size, nd, 4)
            dims = _lib.ame_dims(n, self.r, size, sh.t_begin + off, sh.T_total, self.vcode)
            a = _lib.ame_sweep_args(
                kind=self.group_kinds[size], work_doubles=self._work_half,
                Yt=at(self.Yt, off, nn2, 4), x_old=at(self.xs[src], off, nd, 4),
                x_new=at(self.xs[dst], off, nd, 4), next_old=g_next_old,
                hand=at(self.hand, off, nd, 8), halo_in=g_halo_in, halo_out=g_halo_out,
                cov=at(self.covs[src], off, ndd, 4), consts=_ptr(self.consts),
                rinv=self.C.rinv4(), lr=self.lr, one_minus_lr=float(1.0 - self.lr),
                epoch=self.epoch, status=_ptr(self.status),
                work=at(self.sweep_work, par, self._work_half, 8),
                cov_new=at(self.covs[dst], off, ndd, 4), done=at(self.done, off, 1, 4),
                wait_epoch=wait, back_out=back_out if g == 0 else None,
                back_in=back_in if g == last else None,
                flags=(_lib.AME_SWEEP_FLAG_NEXT_GROUP if g < last else 0)
                | (_lib.AME_SWEEP_FLAG_PREV_GROUP if g > 0 else 0))
            _lib.check(self.L.ame_sweep(ctypes.byref(dims), ctypes.byref(a),
                                        ctypes.c_void_p(stream.cuda_stream)), "ame_sweep")
        self._toc(tok, stream)
        # the kernels take raw pointers: tell the caching allocator these streams
        # use the buffers, so a dropped engine's memory is not handed out again
        # while a sweep still reads or writes it
        done = []
        for st in used:
            for t in (self.xs[src], self.xs[dst], self.covs[src], self.covs[dst], self.hand,
                      self.done, self.status, self.sweep_work, self.Yt, self.consts):
                t.record_stream(st)
            ev = torch.cuda.Event()
            ev.record(st)
            done.append(ev)
        return done, dst

    def _commit(self, slot):
        self._cur = slot
        self._out_valid = False
        self._cov_terms_valid = False

    def sweep(self):
        """One Gauss-Seidel sweep + covariance update (reference _update_step).
        A sweep already started from this state (speculate) is only committed."""
        if self._specs:
            done, slot = self._specs.popleft()
        else:
            done, slot = self._launch_sweep()
        for ev in done:
            self.stream.wait_event(ev)
        self._commit(slot)
        if self.halo is not None:
            self.halo.after_sweep(self)

    def speculate(self, ahead=1):
        """Keep min(ahead, spec_depth) sweeps started beyond the current state.
        Each reads the previous one's output ring slot; none touches the current
        state, and the oldest slot it overwrites belongs to a state whose ELBO
        the host has already read."""
        if not self.speculation:
            return
        want = min(int(ahead), self.spec_depth)
        while len(self._specs) < want:
            self._specs.append(self._launch_sweep(spec=True))

    def discard_speculation(self):
        """Drop started sweeps that will not be committed.  They write only
        spare ring slots; later main-stream work is ordered after them."""
        while self._specs:
            done, _ = self._specs.popleft()
            for ev in done:
                self.stream.wait_event(ev)

    def refresh_cov_terms(self):
        """Covariance ELBO terms of the current covariances (no update)."""
        c = _lib.ame_cov_args(cov=_ptr(self.cov), consts=_ptr(self.consts),
                              cov_terms=_ptr(self.cov_terms))
        st = self._elbo_stream_begin()
        tok = self._tic("cov", st)
        _lib.check(self.L.ame_cov(ctypes.byref(self.dims), ctypes.byref(c),
                                  ctypes.c_void_p(st.cuda_stream)), "ame_cov")
        self._toc(tok)
        self._elbo_stream_end(st)
        self._cov_terms_valid = True

    def launch_elbo(self, pairs_only=False):
        """The ELBO / MSE sums of the current state into self.out.  pairs_only
        (diagnostic timing): the pair kernel alone through ame_elbo_pairs_diag,
        which writes no sums."""
        if not pairs_only and not getattr(self, "_cov_terms_valid", False):
            self.refresh_cov_terms()
        prev_final = None
        if self.halo is not None and not pairs_only:
            prev_final = self.halo.prev_final(self)
        e = _lib.ame_elbo_args(
            Yt=_ptr(self.Yt), x=_ptr(self.x_a), prev_final=prev_final,
            cov_terms=_ptr(self.cov_terms), consts=_ptr(self.consts), phi=_ptr(self.phi),
            rinv=self.C.rinv4(), swap_consistent=1 if self.swap_consistent else 0,
            work=_ptr(self.work), out=_ptr(self.out), pairs_kernel=self.options.pairs_kernel)
        st = self._elbo_stream_begin()
        sp = ctypes.c_void_p(st.cuda_stream)
        if pairs_only:
            tok = self._tic("pairs", st)
            _lib.check(self.L.ame_elbo_pairs_diag(ctypes.byref(self.dims), ctypes.byref(e), sp),
                       "ame_elbo_pairs_diag")
            self._toc(tok)
            self._elbo_stream_end(st)
            return
        tok = self._tic("elbo", st)
        _lib.check(self.L.ame_elbo(ctypes.byref(self.dims), ctypes.byref(e), sp), "ame_elbo")
        self._toc(tok)
        self._elbo_stream_end(st)

    def sums(self, speculate=0):
        """The 8 fp64 sums for the current state (all ranks reduced).  With
        speculate=k > 0 (iterations still to come) up to k next sweeps are
        started first and run beside them."""
        if not self._out_valid:
            if self.elbo_first:
                # the sweep's `ready` event (main stream) then follows the ELBO
                self.launch_elbo()
                if speculate:
                    self.speculate(int(speculate))
            else:
                if speculate:
                    self.speculate(int(speculate))
                self.launch_elbo()
            out = self.out
            if self.halo is not None:
                out = self.halo.allreduce_sums(out)
            self._out_host = out.cpu().tolist()
            self._check_status()
            self._out_valid = True
        return self._out_host

    def terms(self, speculate=0):
        return assemble(self.sums(speculate), self.n, self.T, self.d, self.variant, self.C)

    def _check_status(self):
        words = self.status.cpu().tolist()
        if words[0]:
            self.status.zero_()
            # a later pipelined launch must not start before this zero lands (it
            # would erase that sweep's own status bits)
            self._mark_host_writes()
            self.last_status = words
            raise RuntimeError(f"ame_amd: sweep reported {status_report(words)}")

    def invalidate(self):
        self._out_valid = False
        self._cov_terms_valid = False

    # ------------------------------------------------------------------
    # state transfer (reference layout (n, T, d[, d]))
    # ------------------------------------------------------------------
    def means_local(self) -> torch.Tensor:
        return self.x_a.permute(1, 0, 2)

    def covs_local(self) -> torch.Tensor:
        return self.cov.permute(1, 0, 2, 3)

    def set_means(self, X_mean: torch.Tensor):
        self.discard_speculation()
        sh = self.shard
        t0, t1 = sh.t_begin, sh.t_begin + sh.T_local
        self.x_a.copy_(X_mean[:, t0:t1].detach().float().permute(1, 0, 2))
        self._mark_host_writes()
        self.invalidate()

    def set_covs(self, X_cov: torch.Tensor):
        self.discard_speculation()
        sh = self.shard
        t0, t1 = sh.t_begin, sh.t_begin + sh.T_local
        self.cov.copy_(X_cov[:, t0:t1].detach().float().permute(1, 0, 2, 3))
        self._mark_host_writes()
        self.invalidate()
