"""GPU-backed temporal VI: state lives in HBM, the reference-visible attributes
(``X_mean (n,T,d)``, ``X_cov (n,T,d,d)``, CPU fp32) are lazily synchronised views.

Synchronisation rule: after a device step the device copy is authoritative;
reading ``vi.X_mean`` downloads it once, INTO the host tensor handed out
before (so a reference a caller kept, ``X = vi.X_mean``, sees the fitted
values once the attribute has been read again, like the reference's live
tensor), and remembers the tensor's version counter.  Assigning
``vi.X_mean = ...`` or mutating the host tensor in place (which bumps
``tensor._version``) makes the host copy authoritative again and it is
uploaded before the next device step.

Time-sharded runs: reading ``X_mean`` / ``X_cov`` after a device step is a
COLLECTIVE (every rank's slices are all-gathered), so every rank must read
it, e.g. not only ``if rank == 0``.  ``local_means()`` / ``local_covs()``
return this rank's own slices without communication.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from .base import BaseTemporalVariationalInference
from ..engine import DeviceEngine, EngineOptions


def default_device():
    if not torch.cuda.is_available():
        return None
    lr = os.environ.get("LOCAL_RANK")
    if lr is not None and torch.cuda.device_count() > 1:
        return torch.device("cuda", int(lr) % torch.cuda.device_count())
    return torch.device("cuda", torch.cuda.current_device())


class DeviceTemporalVI(BaseTemporalVariationalInference):
    _variant = "good"

    def __init__(self, model, learning_rate, seed, device=None, distributed=None,
                 engine_options=None):
        self._device = device
        self._distributed = distributed
        self._engine_options = EngineOptions.coerce(engine_options)
        self._engine: Optional[DeviceEngine] = None
        self._host = {"mean": None, "cov": None}
        self._ver = {"mean": None, "cov": None}
        self._stale = {"mean": False, "cov": False}
        super().__init__(model, learning_rate, seed)

    # ---------------- reference-visible state ----------------
    def _get(self, key):
        eng = self._engine
        if eng is not None and self._stale[key]:
            if key == "mean":
                t = self._gather(eng.means_local(), axis=1)
            else:
                t = self._gather(eng.covs_local(), axis=1)
            h = self._host[key]
            if h is not None and h.shape == t.shape and h.dtype == t.dtype and not h.is_inference():
                # refresh in place: a tensor a caller took earlier (X = vi.X_mean)
                # sees the update, as the reference's live attribute does
                # (structured_mf.py:282-287, 332-338)
                h.copy_(t)
                t = h
            self._host[key] = t
            self._ver[key] = t._version
            self._stale[key] = False
        return self._host[key]

    def _set(self, key, value):
        self._host[key] = value
        self._ver[key] = None     # force upload before the next device step
        self._stale[key] = False

    @property
    def X_mean(self):
        return self._get("mean")

    @X_mean.setter
    def X_mean(self, v):
        self._set("mean", v)

    @property
    def X_cov(self):
        return self._get("cov")

    @X_cov.setter
    def X_cov(self, v):
        self._set("cov", v)

    def _host_dirty(self, key):
        h = self._host[key]
        return (not self._stale[key]) and h is not None and (
            self._ver[key] is None or h._version != self._ver[key])

    # ---------------- engine lifecycle ----------------
    def _make_halo(self):
        import torch.distributed as dist
        use = self._distributed
        if use is None:
            use = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        if not use:
            return None, None
        from ..distributed import TimeShardHalo
        # distributed=True / None: defaults; a dict: TimeShardHalo options (peer_mode)
        halo = TimeShardHalo.create(self.T, **(use if isinstance(use, dict) else {}))
        return halo.shard, halo

    def _ensure_engine(self) -> DeviceEngine:
        if self._engine is None:
            dev = self._device if self._device is not None else default_device()
            shard, halo = self._make_halo()
            self._engine = DeviceEngine(self.model, self._variant, self.lr, self._host["mean"],
                                        self._host["cov"], device=dev, shard=shard, halo=halo,
                                        options=self._engine_options)
            self._ver["mean"] = self._host["mean"]._version
            self._ver["cov"] = self._host["cov"]._version
            self._halo = halo
        else:
            eng = self._engine
            if self._host_dirty("mean"):
                eng.set_means(self._host["mean"])
                self._ver["mean"] = self._host["mean"]._version
            if self._host_dirty("cov"):
                eng.set_covs(self._host["cov"])
                self._ver["cov"] = self._host["cov"]._version
        return self._engine

    def _gather(self, local, axis):
        halo = getattr(self, "_halo", None)
        if halo is None:
            return local.detach().to("cpu").contiguous()
        return halo.gather_time(local, axis)

    # ---------------- hooks ----------------
    def _update_step(self) -> None:
        eng = self._ensure_engine()
        eng.sweep()
        self._stale["mean"] = True
        self._stale["cov"] = True

    # ---------------- fit() hooks: the speculation window ----------------
    def _fit_iteration(self, iteration: int, max_iter: int) -> None:
        # iterations that follow this one unless fit() converges first: that many
        # sweeps may be started ahead (bounded by the engine's spec_depth)
        self._spec_next = max(0, max_iter - 1 - iteration)

    def _fit_end(self, ok: bool = True) -> None:
        self._spec_next = 0
        if self._engine is None:
            return
        halo = getattr(self, "_halo", None)
        if not ok:
            # fit() is raising: the peers may sit in a collective this rank never
            # enters (the ELBO all_reduce, agree()), so no barrier here, and a
            # faulted device must not replace the original exception.  The peer
            # buffers stay mapped until close() at exit.
            try:
                self._engine.discard_speculation()
                if halo is not None:
                    halo.quiesce_local(self._engine)
            except Exception:
                pass
            return
        self._engine.discard_speculation()
        if halo is not None:
            # no rank leaves fit() while a neighbour's dropped sweep may still
            # store into its peer buffers (they are freed at close / exit)
            halo.quiesce(self._engine)

    def _terms(self):
        return self._ensure_engine().terms(speculate=getattr(self, "_spec_next", 0))

    def _compute_elbo(self):
        # the reference returns a 0-d fp32 tensor (python float + fp32 tensors)
        return torch.tensor(self._terms()["elbo"], dtype=torch.float32)

    def _compute_expected_log_likelihood(self):
        return torch.tensor(self._terms()["loglik"], dtype=torch.float32)

    def _compute_log_prior_initial(self):
        return torch.tensor(self._terms()["prior0"], dtype=torch.float32)

    def _compute_log_prior_transitions(self):
        return torch.tensor(self._terms()["trans"], dtype=torch.float32)

    def _compute_entropy(self):
        return torch.tensor(self._terms()["entropy"], dtype=torch.float32)

    def _compute_reconstruction_error(self) -> float:
        return float(self._terms()["recon"])

    def elbo_terms(self) -> dict:
        """fp64 ELBO pieces + MSE of the current state (extension)."""
        return dict(self._terms())

    def local_means(self) -> torch.Tensor:
        """This rank's slices (n, T_local, d) of the current means, on the CPU,
        without a collective (extension; equals X_mean on one process)."""
        return self._ensure_engine().means_local().detach().to("cpu").contiguous()

    def local_covs(self) -> torch.Tensor:
        """This rank's slices (n, T_local, d, d) of the current covariances."""
        return self._ensure_engine().covs_local().detach().to("cpu").contiguous()

    def get_variational_means(self) -> torch.Tensor:
        return self.X_mean

    def get_variational_covariances(self) -> torch.Tensor:
        return self.X_cov

    @property
    def engine(self) -> DeviceEngine:
        return self._ensure_engine()
