"""Process-group plumbing: one process per GPU, ``torch.distributed`` over RCCL (backend "nccl"
is RCCL on ROCm) for device tensors, gloo for the CPU test-suite.

Collectives used by the engine:
  X01 all_reduce(int32 Δn_wk ‖ Δn_k)     every sweep          -> :meth:`Comm.allreduce_`
  X02 all_gather(unique word keys)        once (vocabulary)    -> :meth:`Comm.allgather_var`
  X03 all_reduce(radix histograms)        once per cut pass    -> :meth:`Comm.allreduce_np`
  X04 all_reduce(log-likelihood)          every eval           -> :meth:`Comm.allreduce_`
  X05 all_gather(θ rows) for scoring      once                 -> :meth:`Comm.allgather_var`
  X06 all_gather(top-N candidates)        once                 -> :meth:`Comm.allgather_var`
  plus token routing to document owners   once                 -> :meth:`Comm.alltoallv`

The reference used MPI reduce+bcast of K×V doubles per EM iteration and Spark shuffles; here the
per-sweep payload is one int32 buffer and everything else happens once per run.
"""
from __future__ import annotations

import datetime
import os

import numpy as np
import torch
import torch.distributed as dist


class _Pending:
    """An issued async collective: ``wait()`` joins it to the current stream, then runs ``after``."""

    def __init__(self, work, after):
        self.work, self.after = work, after

    def wait(self) -> None:
        self.work.wait()
        if self.after is not None:
            self.after()


class Comm:
    def __init__(self, rank: int = 0, world: int = 1, device: torch.device | None = None, group=None,
                 forced: bool = False, backend: str | None = None):
        self.rank = rank
        self.world = world
        self.device = device or torch.device("cpu")
        self.group = group
        self.backend = backend or ("nccl" if self.device.type == "cuda" else "gloo")
        # gloo over device tensors (ONI_DIST_BACKEND=gloo: several ranks sharing one GPU, the
        # SURVEY §4.3 shard emulation): collectives go through host copies
        self._via_host = self.device.type == "cuda" and self.backend == "gloo"
        # collectives run whenever a process group exists: world > 1, or a forced 1-rank group
        # (ONI_FORCE_DIST=1) that drives the real RCCL / gloo code paths on a single device
        self.dist = world > 1 or forced
        # ONI_COMM_REAL=1: a forced 1-rank group runs every collective for real (one RCCL kernel
        # each: X01 inside the captured sweep graph, the routing all-to-all, the vocabulary and
        # result gathers, the X03 histogram all-reduce) instead of taking the identity shortcut --
        # the hardware rehearsal of the data-parallel path on one GPU. Off (default): a 1-rank
        # group's collectives are the identity (no copy, no launch), as in the overhead bench.
        self.real = self.dist and world == 1 and os.environ.get("ONI_COMM_REAL", "0") == "1"
        # do collectives move data? (several ranks, or a forced-real 1-rank group)
        self.live = self.dist and (world > 1 or self.real)

    # -- basic ------------------------------------------------------------------------------------
    # A 1-rank group (ONI_FORCE_DIST=1) reduces, broadcasts and gathers as the identity unless
    # ONI_COMM_REAL=1 (``live``; on RCCL through a self all-to-all, see _one_rank_rccl): the
    # data-parallel code paths around the collectives run, the collectives themselves do not --
    # as in the sweeps' X01 (models/gibbs.py _allreduce_dn).
    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.live:
            if self._one_rank_rccl():
                return self._reduce_one_rank(t)
            rop = self._rop(op)
            if self._via_host and t.is_cuda:
                h = t.cpu()
                dist.all_reduce(h, op=rop, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=rop, group=self.group)
        return t

    def allreduce_async_(self, t: torch.Tensor):
        """Start a SUM all-reduce of ``t`` in place; returns a handle whose ``wait()`` makes the
        current stream wait for it (RCCL: the process group's own stream runs the collective after
        the work already queued on the current stream, so kernels queued between this call and
        ``wait()`` overlap it -- also inside a HIP graph capture; gloo: wait() blocks). None when
        no collective runs (``wait`` on None: nothing to do)."""
        if not self.live:
            return None
        if self._one_rank_rccl():
            out = self._a2a_scratch(t, "async")  # its own buffer: sync reductions may run before wait()
            work = dist.all_to_all_single(out, t.reshape(-1), group=self.group, async_op=True)
            return _Pending(work, lambda: t.copy_(out.view(t.shape)))
        if self._via_host and t.is_cuda:
            self.allreduce_(t)  # through host copies: synchronous
            return None
        return _Pending(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True), None)

    def _a2a_scratch(self, t: torch.Tensor, tag: str = "sync") -> torch.Tensor:
        key = (t.numel(), t.dtype, tag)
        cache = self.__dict__.setdefault("_a2a_scratch_bufs", {})
        if key not in cache:
            cache[key] = torch.empty(t.numel(), dtype=t.dtype, device=t.device)
        return cache[key]

    def _rop(self, op: str):
        return {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]

    def _one_rank_rccl(self) -> bool:
        """A forced-real 1-rank RCCL group (ONI_COMM_REAL=1, one GPU)? RCCL runs an in-place
        1-rank all-reduce as a no-op -- no kernel, nothing for a graph to hold -- so such a group
        reduces through a self all-to-all (Σ over one rank = the rank's own buffer), which RCCL
        executes as a real p2p kernel over the whole payload: the sweep graph then captures and
        replays an RCCL kernel of the X01 payload's size, joined to the compute stream as a ring
        all-reduce's would be."""
        return self.real and self.backend == "nccl" and self.device.type == "cuda" and not self._via_host

    def _reduce_one_rank(self, t: torch.Tensor) -> torch.Tensor:
        out = self._a2a_scratch(t)
        dist.all_to_all_single(out, t.reshape(-1), group=self.group)
        t.copy_(out.view(t.shape))
        return t

    def allreduce_np(self, a) -> np.ndarray:
        """Sum over ranks → host array. ``a``: a host array, or a device tensor (reduced where it
        lives -- no host→device copy; the caller's tensor is left unchanged)."""
        if torch.is_tensor(a):
            if not self.live:
                return a.cpu().numpy()
            t = a.to(self._coll_device, copy=True)
            self.allreduce_(t)
            return t.cpu().numpy()
        a = np.asarray(a)
        if not self.live:
            return a
        # a private copy: on CPU collectives torch.from_numpy would alias (and reduce into) ``a``
        t = self._small_tensor(a) if a.size == 1 else torch.from_numpy(np.array(a, copy=True)).to(self._coll_device)
        self.allreduce_(t)
        return t.cpu().numpy().reshape(a.shape)

    allreduce_np.accepts_tensors = True  # quantile_cuts hands it device histograms

    def _small_tensor(self, a) -> torch.Tensor:
        """A 1-element collective buffer written by a fill kernel rather than a host→device copy:
        while the next day's columns stream in on the copy engine (io.staging.Prefetcher) a small
        pageable upload queues behind them (measured: ~10 ms of a forced 1-rank day)."""
        a = np.asarray(a)
        return torch.full((1,), a.reshape(-1)[0].item(), dtype=torch.from_numpy(a[:0].reshape(0)).dtype,
                          device=self._coll_device)

    def allreduce_scalar(self, x: float, op: str = "sum") -> float:
        if not self.live:
            return float(x)
        t = torch.full((1,), float(x), dtype=torch.float64, device=self._coll_device)
        self.allreduce_(t, op)
        return float(t.item())

    def barrier(self) -> None:
        if self.dist:
            if self.device.type == "cuda" and self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index or 0])
            else:
                dist.barrier(group=self.group)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.live:
            if self._via_host and t.is_cuda:
                h = t.cpu()
                dist.broadcast(h, src=src, group=self.group)
                t.copy_(h)
            else:
                dist.broadcast(t, src=src, group=self.group)
        return t

    def graph_capturable(self) -> bool:
        """Can this communicator's device collectives be captured into a HIP graph? (RCCL on
        device tensors: yes; gloo, including gloo-through-host-copies: no.)"""
        return self.device.type == "cuda" and self.backend == "nccl" and not self._via_host

    @property
    def _coll_device(self) -> torch.device:
        return torch.device("cpu") if self._via_host else self.device

    # -- variable-size gathers / exchanges ------------------------------------------------------
    def allgather_var(self, t: torch.Tensor) -> list[torch.Tensor]:
        """All-gather tensors whose first dim differs per rank."""
        if not self.live:
            # a 1-rank group (ONI_FORCE_DIST=1) gathers its own tensor: no copy, no collective
            return [t.to(self.device) if self.dist else t]
        if self._via_host and t.is_cuda:
            return [o.to(self.device) for o in self._host_view().allgather_var(t.cpu())]
        n = torch.full((1,), t.shape[0], dtype=torch.int64, device=self.device)
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(ns, n, group=self.group)
        sizes = torch.cat(ns).tolist()  # one device read for all ranks' sizes
        m = max(sizes)
        pad = torch.zeros((m, *t.shape[1:]), dtype=t.dtype, device=self.device)
        pad[: t.shape[0]] = t.to(self.device)
        outs = [torch.zeros_like(pad) for _ in range(self.world)]
        dist.all_gather(outs, pad, group=self.group)
        return [o[:s] for o, s in zip(outs, sizes)]

    def alltoallv(self, t: torch.Tensor, send_counts, recv_counts=None, return_recv_counts: bool = False):
        """Exchange rows: rows [off_r, off_r + send_counts[r]) of ``t`` go to rank r.

        ``recv_counts`` (when the caller already knows them, e.g. the way back of a routed
        exchange) skips the count exchange. ``return_recv_counts`` also returns them (list)."""
        if not self.live:
            # 1-rank group: the exchange is the identity (every row stays) -- no copy, no collective
            if self.dist:
                t = t.to(self.device)
            return (t, [int(t.shape[0])]) if return_recv_counts else t
        sc = [int(x) for x in (send_counts.tolist() if torch.is_tensor(send_counts) else send_counts)]
        if self._via_host and t.is_cuda:
            r = self._host_view().alltoallv(t.cpu(), sc, recv_counts, return_recv_counts)
            return (r[0].to(self.device), r[1]) if return_recv_counts else r.to(self.device)
        if recv_counts is None:
            sct = torch.tensor(sc, dtype=torch.int64, device=self.device)
            rct = torch.empty_like(sct)
            dist.all_to_all_single(rct, sct, group=self.group)
            rc = rct.tolist()
        else:
            rc = [int(x) for x in recv_counts]
        out = torch.empty((sum(rc), *t.shape[1:]), dtype=t.dtype, device=self.device)
        dist.all_to_all_single(out, t.to(self.device).contiguous(), output_split_sizes=rc,
                               input_split_sizes=sc, group=self.group)
        return (out, rc) if return_recv_counts else out

    def host_side(self) -> "Comm":
        """A CPU communicator on a process group of its own (gloo), for host-side collectives
        issued from a worker thread (the multi-day loader's IPv6 dictionary exchange) while the
        main thread drives the device collectives: two groups, so the two threads' collectives
        never interleave on one channel. Collective call: every rank creates it in the same order."""
        if getattr(self, "_host_side", None) is None:
            if not self.dist:
                self._host_side = Comm(self.rank, self.world, torch.device("cpu"), backend="gloo")
            else:
                g = dist.new_group(backend="gloo")
                self._host_side = Comm(self.rank, self.world, torch.device("cpu"), g, forced=True, backend="gloo")
        return self._host_side

    def side_group(self, name: str) -> "Comm":
        """A further CPU (gloo) communicator of its own, for one more worker thread's host-side
        collectives (e.g. the result pipe's rendered-row gather) -- like :meth:`host_side`, each
        thread owns its group so no two threads' collectives interleave on one channel.
        Collective call: every rank creates it in the same order."""
        groups = self.__dict__.setdefault("_side_groups", {})
        if name not in groups:
            if not self.dist:
                groups[name] = Comm(self.rank, self.world, torch.device("cpu"), backend="gloo")
            else:
                g = dist.new_group(backend="gloo")
                groups[name] = Comm(self.rank, self.world, torch.device("cpu"), g, forced=True, backend="gloo")
        return groups[name]

    def _host_view(self) -> "Comm":
        v = Comm(self.rank, self.world, torch.device("cpu"), self.group, forced=self.dist, backend="gloo")
        v.real, v.live = self.real, self.live
        return v

    def agree(self, ok: bool) -> bool:
        """Rank-consistent vote: True on every rank iff ``ok`` on every rank (an eager MIN
        all-reduce; the identity without a process group). Used after a HIP-graph capture of the
        sweeps (models/gibbs.py): one rank's failed capture sends every rank to eager sweeps."""
        if not self.live:
            return bool(ok)
        t = torch.full((1,), 1 if ok else 0, dtype=torch.int32, device=self._coll_device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(t.item()))


def init_from_env(device_type: str | None = None, timeout_s: float = 600.0) -> Comm:
    """Initialise from torchrun env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); world 1 if absent."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    # ONI_DIST_BACKEND=gloo with device tensors: several ranks may share one GPU (shard emulation,
    # SURVEY §4.3) -- ranks map onto the visible devices round-robin; RCCL needs one GPU per rank
    backend = os.environ.get("ONI_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    if device_type == "cuda" and backend == "gloo":
        local %= max(torch.cuda.device_count(), 1)
    device = torch.device(device_type, local) if device_type == "cuda" else torch.device("cpu")
    if device_type == "cuda":
        torch.cuda.set_device(device)
    forced = os.environ.get("ONI_FORCE_DIST", "0") == "1"
    if world == 1 and not forced:
        return Comm(0, 1, device)
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if not dist.is_initialized():
        kw = {}
        if device_type == "cuda" and backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return Comm(rank, world, device, forced=forced, backend=backend)


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
