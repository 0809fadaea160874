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
  sweep lane writes {epoch,value} granules into a host-shared buffer that both
  processes map (hipHostRegister), and rank g's first lane polls them.  No
  collective sits on the data path; the wavefront simply continues across the
  GPU boundary;
* after the sweep: all_gather of last-slice means (the transition term of the
  ELBO at t_begin) and an fp64 all_reduce of the 8 ELBO/MSE sums;
* pipelined sweeps (the next sweep queued while this one runs): the right halo
  cannot come from a collective, so each rank's first slice also writes its
  final means into a back channel in the same shared buffer when it finishes
  (system-scope release + done word), and the left rank's last slice of the
  next sweep waits for that word instead.

``shard_range`` / ``assemble``-level logic is exercised on CPU by
tests/test_distributed_cpu.py (gloo, world_size 2).
"""
from __future__ import annotations

import atexit
import ctypes
import mmap
import os
import uuid
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


class HostHalo:
    """A granule buffer in /dev/shm, pinned and mapped for device access."""

    def __init__(self, path: str, nbytes: int, create: bool):
        self.path, self.nbytes = path, nbytes
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, nbytes)
            self.mm = mmap.mmap(fd, nbytes, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        if create:
            self.mm[:] = bytes(nbytes)
        self._cbuf = (ctypes.c_char * nbytes).from_buffer(self.mm)
        self.host = ctypes.c_void_p(ctypes.addressof(self._cbuf))
        dev = ctypes.c_void_p()
        _lib.check(_lib.lib().ame_host_register(self.host, nbytes, ctypes.byref(dev)),
                   "ame_host_register")
        self.dev = dev
        self.owner = create

    def close(self):
        if self.mm is None:
            return
        try:
            _lib.lib().ame_host_unregister(self.host)
        except Exception:
            pass
        self.host = None
        self._cbuf = None
        try:
            self.mm.close()
        except BufferError:
            pass
        self.mm = None
        if self.owner:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


class TimeShardHalo:
    """Halo exchange for one engine (rank) of a time-sharded run."""

    def __init__(self, shard: Shard, group=None):
        self.shard = shard
        self.group = group
        self.left: Optional[HostHalo] = None
        self.right: Optional[HostHalo] = None
        self._next_old = None
        self._prev_final = None
        # gloo (CPU tests, several ranks sharing one GPU) needs host staging
        self._host_coll = dist.get_backend(group) == "gloo"

    def _coll(self, t: torch.Tensor):
        return t.cpu() if (self._host_coll and t.is_cuda) else t

    @classmethod
    def create(cls, T: int, group=None) -> "TimeShardHalo":
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        t0, tl = shard_range(T, world, rank)
        return cls(Shard(t0, tl, T, rank, world), group)

    # ---- setup (called once the engine knows n, d) ----
    def _setup(self, eng):
        if self.left is not None or self.right is not None or self.shard.world == 1:
            return
        tag = [uuid.uuid4().hex[:12] if self.shard.rank == 0 else None]
        dist.broadcast_object_list(tag, src=0, group=self.group)
        nd = eng.n * eng.d
        self._back_off = nd * 8                                    # after the granules
        nbytes = max(4096, self._back_off + (((nd + 63) // 64) * 64 + 64) * 4)
        rank, world = self.shard.rank, self.shard.world
        base = f"/dev/shm/ame_halo_{tag[0]}"
        if rank > 0:   # consumer of boundary (rank-1 -> rank) creates it
            self.left = HostHalo(f"{base}_{rank - 1}", nbytes, create=True)
        dist.barrier(group=self.group)
        if rank < world - 1:
            self.right = HostHalo(f"{base}_{rank}", nbytes, create=False)
        dist.barrier(group=self.group)
        atexit.register(self.close)

    def close(self):
        for h in (self.left, self.right):
            if h is not None:
                h.close()
        self.left = self.right = None

    def _all_gather_slice(self, t: torch.Tensor):
        src = self._coll(t.contiguous())
        out = [torch.empty_like(src) for _ in range(self.shard.world)]
        dist.all_gather(out, src, group=self.group)
        return [o.to(t.device) for o in out]

    # ---- engine hooks ----
    def agree(self, eng, flag: bool) -> bool:
        """True only if every rank passes True."""
        t = torch.tensor([1 if flag else 0], dtype=torch.int32,
                         device="cpu" if self._host_coll else eng.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(t.item())

    def back_channels(self, eng):
        """(back_in, back_out) device addresses: the right boundary's back channel
        is read by this rank's last slice, the left one written by its first."""
        self._setup(eng)
        back_in = back_out = None
        if self.right is not None:
            back_in = ctypes.c_void_p(self.right.dev.value + self._back_off)
        if self.left is not None:
            back_out = ctypes.c_void_p(self.left.dev.value + self._back_off)
        return back_in, back_out

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
        halo_in = self.left.dev if self.left is not None else None
        halo_out = self.right.dev if self.right is not None else None
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
