"""Time-sharded multi-GPU execution of the VI sweep (one process per GPU).

Partitioning: contiguous blocks of time slices per rank.  The
observation terms at time t use only time-t data, so Y, the slice's node means
and its running statistics are rank-local.  Ranks couple only through the AR(1)
terms of the boundary slices (structured_mf.py:255-264):

* right halo, OLD means of slice t_end (first slice of rank g+1) -- pre-sweep
  values: one RCCL all_gather of every rank's first-slice means before the
  sweep;
* left halo, NEW means of slice t_begin-1 (last slice of rank g-1) -- produced
  node by node DURING the same sweep (exact Gauss-Seidel order): rank g-1's last
  sweep lane stores {epoch,value} granules with system-scope stores straight
  into a buffer in rank g's HBM (xGMI peer write), and rank g's first lane polls
  its local copy.  No collective and no host memory sit on the data path; the
  wavefront simply continues across the GPU boundary;
* after the sweep: all_gather of last-slice means (the transition term of the
  ELBO at t_begin) and an fp64 all_reduce of the 8 ELBO/MSE sums;
* pipelined sweeps (the next sweep queued while this one runs): the right halo
  cannot come from a collective, so each rank's first slice also writes its
  final means into a back channel in rank g-1's HBM when it finishes
  (system-scope release + done word), and rank g-1's last slice of the next
  sweep waits for that word instead.

Every peer buffer lives on the GPU that POLLS it (fine-grained device memory,
exported with an IPC handle, ame_peer_alloc / ame_peer_open); the neighbour
only writes into it.  The handles travel over the process group.  All ranks
must be on one node (xGMI); that is checked at setup.

``shard_range`` / ``assemble``-level logic is exercised on CPU by
tests/test_distributed_cpu.py (gloo, world_size 2); the peer buffers by
tests/test_gpu_distributed.py (2-4 processes on one GPU: same-device IPC).
"""
from __future__ import annotations

import atexit
import ctypes
import os
import socket
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from . import _lib
from .engine import Shard


def shard_range(T: int, world: int, rank: int) -> Tuple[int, int]:
    """Balanced contiguous split of T slices over `world` ranks -> (t_begin, T_local)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} / world {world}")
    if T < world:
        raise ValueError(f"cannot shard T={T} time steps over {world} ranks")
    base, extra = divmod(T, world)
    t_begin = rank * base + min(rank, extra)
    return t_begin, base + (1 if rank < extra else 0)


class PeerBuffer:
    """Fine-grained device memory: owned (allocated here, exported) or mapped
    (opened from a neighbour's handle)."""

    def __init__(self, nbytes: int = 0, handle: Optional[bytes] = None):
        L = _lib.lib()
        self.dev = ctypes.c_void_p()
        if handle is None:
            h = (ctypes.c_char * _lib.AME_PEER_HANDLE_BYTES)()
            _lib.check(L.ame_peer_alloc(nbytes, ctypes.byref(self.dev), h), "ame_peer_alloc")
            self.handle = bytes(h)
            self.owner = True
        else:
            h = (ctypes.c_char * _lib.AME_PEER_HANDLE_BYTES).from_buffer_copy(handle)
            _lib.check(L.ame_peer_open(h, ctypes.byref(self.dev)), "ame_peer_open")
            self.handle = handle
            self.owner = False

    def close(self):
        if self.dev is None or not self.dev.value:
            return
        try:
            L = _lib.lib()
            (L.ame_peer_free if self.owner else L.ame_peer_close)(self.dev)
        except Exception:
            pass
        self.dev = None


class HostPeerBuffer:
    """The host-memory form of a peer buffer: a POSIX shared-memory file
    (/dev/shm) mapped into each process and registered for device access
    (ame_host_register: hipHostRegister, mapped + portable), so the neighbour's
    system-scope stores and this rank's system-scope polls meet in host memory
    instead of in the owner's HBM.  The fallback when the device-IPC peer link
    fails its pre-flight (TimeShardHalo peer_mode "auto"); slower per poll
    (host memory over the fabric), same protocol, same results."""

    def __init__(self, nbytes: int = 0, handle=None):
        import mmap
        import uuid
        L = _lib.lib()
        self.dev = ctypes.c_void_p()
        if handle is None:
            name = f"/dev/shm/ame_amd_{os.getpid()}_{uuid.uuid4().hex[:12]}"
            fd = os.open(name, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
            os.ftruncate(fd, nbytes)      # zero-filled
            self.owner = True
        else:
            name, nbytes = handle
            fd = os.open(name, os.O_RDWR)
            self.owner = False
        try:
            self._mm = mmap.mmap(fd, nbytes)
        finally:
            os.close(fd)
        self._path, self._bytes = name, nbytes
        self._cbuf = (ctypes.c_char * nbytes).from_buffer(self._mm)
        self._host = ctypes.c_void_p(ctypes.addressof(self._cbuf))
        try:
            _lib.check(L.ame_host_register(self._host, nbytes, ctypes.byref(self.dev)),
                       "ame_host_register")
        except Exception:
            self._release(register=False)
            raise
        self.handle = (name, nbytes)

    def _release(self, register=True):
        if register:
            try:
                _lib.lib().ame_host_unregister(self._host)
            except Exception:
                pass
        self._cbuf = None
        try:
            self._mm.close()
        except Exception:
            pass
        if self.owner:
            try:
                os.unlink(self._path)
            except OSError:
                pass

    def close(self):
        if self.dev is None:
            return
        self._release()
        self.dev = None


class TimeShardHalo:
    """Halo exchange for one engine (rank) of a time-sharded run.

    peer_mode: "ipc" -- the peer buffers live in the polling rank's HBM and the
    neighbour maps them over device IPC (xGMI stores); "host" -- POSIX shared
    host memory registered on both devices (HostPeerBuffer); "auto" (default)
    -- ipc, and host when the ipc links fail their pre-flight on any rank (every
    rank then switches, so all ranks use one mode)."""

    PEER_MODES = ("auto", "ipc", "host")

    def __init__(self, shard: Shard, group=None, peer_mode: str = "auto"):
        if peer_mode not in self.PEER_MODES:
            raise ValueError(f"peer_mode must be one of {self.PEER_MODES}, got {peer_mode!r}")
        self.shard = shard
        self.group = group
        self.peer_mode = peer_mode
        self.peer_kind = None    # "ipc" or "host" once the links passed their pre-flight
        self.preflight_log = []  # failures of a mode that was given up ("auto")
        self._peers = None       # (own halo, own back, peer halo, peer back) PeerBuffers
        self._next_old = None
        self._prev_final = None
        # gloo (CPU tests, several ranks sharing one GPU) needs host staging
        self._host_coll = dist.get_backend(group) == "gloo"
        self.preflight_ok = False    # set by _preflight once every peer link carried its sentinel

    def _coll(self, t: torch.Tensor):
        return t.cpu() if (self._host_coll and t.is_cuda) else t

    @classmethod
    def create(cls, T: int, group=None, peer_mode: str = "auto") -> "TimeShardHalo":
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        t0, tl = shard_range(T, world, rank)
        return cls(Shard(t0, tl, T, rank, world), group, peer_mode)

    # ---- setup (called once the engine knows n, d) ----
    def _setup(self, eng):
        if self._peers is not None or self.shard.world == 1:
            return
        world = self.shard.world
        hosts = [None] * world
        dist.all_gather_object(hosts, socket.gethostname(), group=self.group)
        if len(set(hosts)) != 1:
            raise RuntimeError(
                "ame_amd: time-sharded ranks hand boundary means over xGMI peer memory and "
                f"must all run on one node; got hosts {sorted(set(hosts))}")
        nd = eng.n * eng.d
        self._back_bytes = (((nd + 63) // 64) * 64 + 64) * 4      # floats + done word
        kinds = {"auto": ("ipc", "host"), "ipc": ("ipc",), "host": ("host",)}[self.peer_mode]
        for i, kind in enumerate(kinds):
            try:
                self._setup_kind(eng, kind)
                self.peer_kind = kind
                break
            except Exception as e:   # noqa: BLE001 -- every rank raised alike (pre-flight)
                if i + 1 == len(kinds):
                    raise
                self.preflight_log.append(f"{kind}: {e}")
        atexit.register(self.close)

    def _setup_kind(self, eng, kind: str):
        """Allocate / map the four peer buffers of one kind and pre-flight them.
        Allocation and mapping failures are recorded, not raised, so every rank
        reaches the pre-flight's barrier and all_reduce and raises together."""
        rank, world = self.shard.rank, self.shard.world
        nd = eng.n * eng.d
        Buf = PeerBuffer if kind == "ipc" else HostPeerBuffer
        pre_bad = []

        def make(what, **kw):
            try:
                return Buf(**kw)
            except Exception as e:   # noqa: BLE001 -- reported on every rank by the pre-flight
                pre_bad.append(f"rank {rank}: {kind} {what}: {e}")
                return None
        with torch.cuda.device(eng.dev):
            # buffers this rank POLLS: its left halo (granules from rank-1) and the
            # back channel of its right boundary (final means of rank+1's first slice)
            own_halo = make("left halo", nbytes=nd * 8) if rank > 0 else None
            own_back = make("back channel", nbytes=self._back_bytes) if rank < world - 1 else None
            mine = (own_halo.handle if own_halo else None, own_back.handle if own_back else None)
            allh = [None] * world
            dist.all_gather_object(allh, mine, group=self.group)
            peer_halo = peer_back = None
            if rank < world - 1 and allh[rank + 1][0] is not None:
                peer_halo = make("map of the right rank's halo", handle=allh[rank + 1][0])
            if rank > 0 and allh[rank - 1][1] is not None:
                peer_back = make("map of the left rank's back channel", handle=allh[rank - 1][1])
            if (rank < world - 1 and peer_halo is None) or (rank > 0 and peer_back is None):
                pre_bad.append(f"rank {rank}: {kind}: a neighbour's buffer is missing")
        peers = (own_halo, own_back, peer_halo, peer_back)
        try:
            self._preflight(eng, peers, pre_bad=pre_bad, mode=kind)
        except Exception:
            # nothing may sweep over a link that failed: _peers stays unset, so a
            # caller that catches this and fits again re-runs the setup (and the
            # pre-flight) instead of spinning on the bad link
            for p in peers:
                if p is not None:
                    p.close()
            raise
        self._peers = peers

    @staticmethod
    def _sentinel(kind: int, writer: int, owner: int) -> int:
        # high word 0xA3E5xxxx: never an epoch the sweep waits for (epochs count
        # up from 1), and the buffers are zeroed again after the check
        return ((0xA3E50000 | (kind << 12) | (writer & 0xFFF)) << 32) | (owner & 0xFFFFFFFF)

    def _preflight(self, eng, peers, wait_s: float = 2.0, pre_bad=None, mode: str = "ipc"):
        """Every peer link once, before the first sweep: each rank stores a
        sentinel into each buffer it MAPPED (the right neighbour's halo, the left
        neighbour's back channel) with the same system-scope store the sweep's
        hand-off uses, from its own device; after a barrier every owner reads
        its buffers back.  A missing or wrong value raises naming the rank pair
        and the link, instead of the first sweep spinning until the status word
        reports a halo timeout.  pre_bad: failures of the buffers' allocation /
        mapping (raised here, on every rank alike).  Reference:
        structured_mf.py:240 (the T loop whose boundary the links carry)."""
        import time
        L = _lib.lib()
        rank = self.shard.rank
        own_halo, own_back, peer_halo, peer_back = peers
        bad = list(pre_bad or [])

        def call(fn, *args, what):
            # a library error is recorded, never raised here: every rank must
            # reach the barrier and the all_reduce below, or its peers would wait
            # in them until the process-group timeout
            try:
                _lib.check(fn(*args), what)
                return True
            except Exception as e:   # noqa: BLE001 -- reported on every rank below
                bad.append(f"rank {rank}: {e}")
                return False

        with torch.cuda.device(eng.dev):
            if peer_halo is not None:
                call(L.ame_peer_probe, peer_halo.dev, self._sentinel(1, rank, rank + 1),
                     what=f"ame_peer_probe (rank {rank} -> halo of rank {rank + 1})")
            if peer_back is not None:
                call(L.ame_peer_probe, peer_back.dev, self._sentinel(2, rank, rank - 1),
                     what=f"ame_peer_probe (rank {rank} -> back channel of rank {rank - 1})")
        dist.barrier(group=self.group)
        with torch.cuda.device(eng.dev):
            for buf, writer, kind, nbytes, what in (
                    (own_halo, rank - 1, 1, eng.n * eng.d * 8, "left halo"),
                    (own_back, rank + 1, 2, self._back_bytes, "back channel")):
                if buf is None:
                    continue
                want = self._sentinel(kind, writer, rank)
                got = ctypes.c_ulonglong(0)
                t0 = time.monotonic()
                read_ok = True
                while True:
                    if not call(L.ame_peer_read_u64, buf.dev, ctypes.byref(got),
                                what=f"ame_peer_read_u64 ({what} of rank {rank})"):
                        read_ok = False
                        break
                    if got.value == want or time.monotonic() - t0 > wait_s:
                        break
                    time.sleep(0.01)
                if read_ok and got.value != want:
                    bad.append(f"rank {writer} -> rank {rank} ({what}): read {got.value:#018x}, "
                               f"expected {want:#018x}")
                call(L.ame_peer_clear, buf.dev, nbytes, what=f"ame_peer_clear ({what} of rank {rank})")
        flag = torch.tensor([len(bad)], dtype=torch.int32,
                            device="cpu" if self._host_coll else eng.dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        if bad:
            msg = L.ame_last_error().decode(errors="replace")
            raise RuntimeError(f"ame_amd: peer-link pre-flight ({mode}) failed: " + "; ".join(bad) +
                               f" (last library message: {msg!r})")
        if int(flag.item()):
            raise RuntimeError(f"ame_amd: peer-link pre-flight ({mode}) failed on another rank")
        self.preflight_ok = True

    def quiesce(self, eng):
        """Called by every rank when fit() ends (after the dropped speculative
        sweeps were queued behind): wait for this rank's kernels, then for every
        rank's.  After it no sweep of a neighbour still stores into this rank's
        peer buffers over xGMI, so close() may free them.  Reference: nothing
        (single process)."""
        if self._peers is None:
            return
        torch.cuda.synchronize(eng.dev)
        dist.barrier(group=self.group)

    def close(self):
        """Free / unmap the peer buffers (at exit).  Every fit() ended with
        quiesce(), so no kernel of any rank writes them any more; the local
        synchronize covers a process that leaves without finishing a fit()."""
        if self._peers is None:
            return
        try:
            torch.cuda.synchronize()
        except Exception:
            pass
        for p in self._peers:
            if p is not None:
                p.close()
        self._peers = None

    def _all_gather_slice(self, t: torch.Tensor):
        src = self._coll(t.contiguous())
        out = [torch.empty_like(src) for _ in range(self.shard.world)]
        dist.all_gather(out, src, group=self.group)
        return [o.to(t.device) for o in out]

    def quiesce_local(self, eng):
        """Exception path of fit(): wait for this rank's own kernels only (no
        collective: the other ranks may be inside a different one)."""
        if self._peers is None:
            return
        torch.cuda.synchronize(eng.dev)

    # ---- engine hooks ----
    @staticmethod
    def device_key(dev) -> tuple:
        """Identity of a GPU across processes: host, PCI address and UUID."""
        p = torch.cuda.get_device_properties(dev)
        return (socket.gethostname(), int(getattr(p, "pci_domain_id", 0)),
                int(getattr(p, "pci_bus_id", 0)), int(getattr(p, "pci_device_id", 0)),
                str(getattr(p, "uuid", "")))

    def device_sharers(self, eng) -> int:
        """Number of ranks of the group that run on this rank's GPU (1 on a
        node with one rank per GPU; k when k ranks share one, as the one-GPU
        tests do).  The engine divides its co-resident slice budget by it: a
        spinning launch of any of them may wait on a slice of another
        (DESIGN.md §5).  Reference: none (single process)."""
        if self.shard.world == 1:
            return 1
        if getattr(self, "_sharers", None) is None:
            key = self.device_key(eng.dev)
            keys = [None] * self.shard.world
            dist.all_gather_object(keys, key, group=self.group)
            self._sharers = sum(1 for k in keys if k == key)
        return self._sharers

    def agree_max(self, eng, value: int) -> int:
        """The maximum of `value` over all ranks (the engines' epoch base)."""
        t = torch.tensor([int(value)], dtype=torch.int64,
                         device="cpu" if self._host_coll else eng.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def agree(self, eng, flag: bool) -> bool:
        """True only if every rank passes True."""
        t = torch.tensor([1 if flag else 0], dtype=torch.int32,
                         device="cpu" if self._host_coll else eng.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(t.item())

    def back_channels(self, eng):
        """(back_in, back_out) device addresses: the right boundary's back channel
        (local) is read by this rank's last slice; the left one (rank-1's HBM) is
        written by its first."""
        self._setup(eng)
        if self._peers is None:
            return None, None
        own_halo, own_back, peer_halo, peer_back = self._peers
        return (own_back.dev if own_back else None), (peer_back.dev if peer_back else None)

    def before_sweep(self, eng, gather=True, first=None):
        """first: this rank's first slice of the sweep's input state (the
        current state unless given)."""
        self._setup(eng)
        rank, world = self.shard.rank, self.shard.world
        next_old = None
        if gather:
            firsts = self._all_gather_slice(eng.x_a[0] if first is None else first)
            if rank < world - 1:
                self._next_old = firsts[rank + 1]
                next_old = ctypes.c_void_p(self._next_old.data_ptr())
        halo_in = halo_out = None
        if self._peers is not None:
            own_halo, _, peer_halo, _ = self._peers
            halo_in = own_halo.dev if own_halo else None
            halo_out = peer_halo.dev if peer_halo else None
        return next_old, halo_in, halo_out

    def after_sweep(self, eng):
        self._prev_final = None

    def prev_final(self, eng):
        # collective on every rank (rank 0 discards the result)
        if self._prev_final is None:
            lasts = self._all_gather_slice(eng.x_a[eng.shard.T_local - 1])
            self._prev_final = lasts[self.shard.rank - 1] if self.shard.rank > 0 else lasts[0]
        if self.shard.rank == 0:
            return None
        return ctypes.c_void_p(self._prev_final.data_ptr())

    def allreduce_sums(self, out: torch.Tensor) -> torch.Tensor:
        red = self._coll(out).clone()
        dist.all_reduce(red, op=dist.ReduceOp.SUM, group=self.group)
        return red.to(out.device)

    def gather_time(self, local: torch.Tensor, axis: int) -> torch.Tensor:
        """All ranks' (n, T_local, ...) blocks -> full (n, T, ...) on the CPU."""
        sizes = [shard_range(self.shard.T_total, self.shard.world, r)[1]
                 for r in range(self.shard.world)]
        loc = self._coll(local.contiguous())
        mx = max(sizes)
        if loc.shape[axis] < mx:   # pad to a common shape for all_gather
            pad_shape = list(loc.shape)
            pad_shape[axis] = mx - loc.shape[axis]
            loc = torch.cat([loc, loc.new_zeros(pad_shape)], dim=axis)
        parts = [torch.empty_like(loc) for _ in sizes]
        dist.all_gather(parts, loc, group=self.group)
        parts = [p.narrow(axis, 0, s) for p, s in zip(parts, sizes)]
        return torch.cat(parts, dim=axis).cpu()
