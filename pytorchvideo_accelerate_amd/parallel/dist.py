"""Process-group bootstrap and small collectives (one process per GPU, RCCL over xGMI).

Mirrors what the reference gets from ``accelerate``:

* ``DistState.from_env()`` reads the torchrun / ``accelerate launch`` contract (``RANK``, ``LOCAL_RANK``,
  ``WORLD_SIZE``, ``MASTER_ADDR``, ``MASTER_PORT``); with ``LOCAL_RANK`` set and a GPU present it
  initialises the ``nccl`` backend (RCCL on ROCm) and binds ``cuda:LOCAL_RANK``; on CPU with
  world > 1 it uses ``gloo``; otherwise it is single-process (``distributed_type == "NO"``).
* ``PVA_FORCE_GRADSYNC=1`` initialises the process group even at world size 1 (``multi`` is then true): every
  collective, the gradient all-reduce included, runs through the real backend — RCCL's code paths (``ReduceOp.AVG``,
  ``barrier(device_ids)``, ``all_gather_into_tensor``, the comm-stream bucket schedule) executed on a 1-GPU box
  (SURVEY.md §4.3 item 4).
* ``broadcast_module`` (rank-0 params + buffers, coalesced into one flat buffer per dtype),
  ``all_gather_cat`` (``accelerator.gather``), ``all_reduce_`` (AVG on RCCL, SUM/W on gloo), barrier.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistState:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: Optional[str] = None
    device: torch.device = torch.device("cpu")
    distributed_type: str = "NO"
    forced: bool = False      # PVA_FORCE_GRADSYNC=1: a process group (and every collective) even at world size 1
    comm: Optional[object] = None   # PVA_COMM=rccl: the framework-owned RCCL communicator (parallel/rccl.py)

    @property
    def is_main_process(self) -> bool:
        return self.rank == 0

    @property
    def initialized(self) -> bool:
        return dist.is_available() and dist.is_initialized()

    @property
    def multi(self) -> bool:
        """Collectives are live: a process group with more than one rank, or a forced single-rank group."""
        return self.initialized and (self.world_size > 1 or self.forced)

    @classmethod
    def from_env(cls, cpu: bool = False, timeout_s: int = 1800) -> "DistState":
        ws = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        use_gpu = (not cpu) and torch.cuda.is_available()
        st = cls(rank=rank, world_size=ws, local_rank=lr)
        st.forced = os.environ.get("PVA_FORCE_GRADSYNC", "0") == "1"
        if use_gpu:
            ndev = torch.cuda.device_count()
            st.device = torch.device("cuda", lr % max(ndev, 1))
            torch.cuda.set_device(st.device)
        if ws > 1 or st.forced:
            # PVA_DIST_BACKEND=gloo on a GPU: several ranks may share one device (1-GPU rehearsal of the
            # multi-rank path; RCCL refuses duplicate devices).  Default on GPU: nccl (= RCCL on ROCm).
            st.backend = os.environ.get("PVA_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
            if ws > 1:
                st.distributed_type = "MULTI_GPU" if use_gpu else "MULTI_CPU"
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29500")
                import datetime
                kw = {}
                if use_gpu and st.backend == "nccl":
                    kw["device_id"] = st.device
                    # collectives on a high-priority HIP stream: bucket all-reduces overlapping the
                    # backward pass get scheduled ahead of the compute stream's queued kernels
                    opts = dist.ProcessGroupNCCL.Options()
                    opts.is_high_priority_stream = True
                    kw["pg_options"] = opts
                timeout = datetime.timedelta(seconds=timeout_s)
                if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
                    # under the torchrun agent: join its TCPStore with a per-attempt prefix so an elastic
                    # restart never reads the previous attempt's connection keys (stale gloo/RCCL peers)
                    base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), ws, False,
                                         timeout=timeout)
                    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
                    kw["store"] = dist.PrefixStore(f"pva/attempt_{attempt}/", base)
                dist.init_process_group(st.backend, rank=rank, world_size=ws, timeout=timeout, **kw)
            if use_gpu and st.backend == "nccl" and os.environ.get("PVA_COMM", "pg") == "rccl":
                import atexit
                from .rccl import RcclCommunicator
                st.comm = RcclCommunicator(rank, ws, st.broadcast_object)
                atexit.register(st.comm.close)   # destroyed while the HIP runtime is still up
        return st

    # -------------------------------------------------------------- collectives
    def barrier(self):
        if self.multi:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def agree_times(self, times: List[float]) -> List[float]:
        """Autotuner consensus: every rank times the same candidate list; all pick the argmin of the
        per-candidate MAX over ranks (the slowest rank bounds a data-parallel step), so every rank runs
        identical kernels."""
        if not self.multi or not times:
            return times
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor(times, dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.cpu().tolist()

    def all_reduce_(self, t: torch.Tensor, op: str = "avg") -> torch.Tensor:
        if not self.multi:
            return t
        if op == "avg":
            if self.backend == "nccl":
                dist.all_reduce(t, op=dist.ReduceOp.AVG)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                t.div_(self.world_size)
        elif op == "sum":
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elif op == "max":
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        else:
            raise ValueError(op)
        return t

    def all_gather_cat(self, t: torch.Tensor) -> torch.Tensor:
        """``accelerator.gather``: concatenate every rank's tensor along dim 0 (equal shapes)."""
        if not self.multi:
            return t
        t = t.contiguous()
        if self.backend == "nccl":
            out = torch.empty((self.world_size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t)
            return out
        parts = [torch.empty_like(t) for _ in range(self.world_size)]
        dist.all_gather(parts, t)
        return torch.cat(parts, 0)

    def broadcast_tensors(self, tensors: List[torch.Tensor], src: int = 0):
        """Coalesced broadcast (one flat buffer per dtype) of rank ``src``'s tensors, in place."""
        if not self.multi or not tensors:
            return
        by_dtype = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        for dt, ts in by_dtype.items():
            flat = torch.cat([t.reshape(-1) for t in ts])
            dist.broadcast(flat, src)
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n

    def broadcast_module(self, module: torch.nn.Module, src: int = 0, buffers_only: bool = False):
        ts = [] if buffers_only else [p.data for p in module.parameters()]
        ts += [b for b in module.buffers()]
        self.broadcast_tensors(ts, src)

    def broadcast_object(self, obj, src: int = 0):
        if not self.multi:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src)
        return lst[0]

    def destroy(self):
        if self.initialized:
            dist.destroy_process_group()
