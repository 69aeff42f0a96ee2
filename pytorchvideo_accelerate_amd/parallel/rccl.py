"""Framework-owned RCCL communicator (native part: csrc/runtime/rccl_comm.cpp).

``PVA_COMM=rccl`` makes the gradient all-reduce (``parallel/ddp.GradSync``) bypass torch's ProcessGroupNCCL: one
``ncclComm_t`` per process, created from a unique id that rank 0 makes and the bootstrap process group broadcasts,
and every bucket's ``ncclAllReduce(avg)`` enqueued directly on the executor's own communication stream (the one that
already waits on every gradient-producing stream by events).  Completion is an event recorded after the collective on
that stream, which the compute stream waits on in ``finish()`` — no Work objects, no internal PG stream, no extra
event hop per bucket.  The rest of the control plane (barriers, object broadcasts, metric gathers) stays on the
process group, which also carries the bootstrap.

The library is torch's own ``lib/librccl.so`` bound at run time (a second, link-time RCCL in the same process
corrupted the first one's state); ``PVA_RCCL_LIB`` overrides the path.
"""
from __future__ import annotations

import os
from typing import Optional

import torch


def torch_rccl_path() -> str:
    return os.environ.get("PVA_RCCL_LIB") or os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


class EventWork:
    """``Work``-like handle of a collective enqueued on a stream: ``wait()`` makes the current stream wait for it."""

    def __init__(self, stream: Optional[torch.cuda.Stream] = None):
        self.event = torch.cuda.Event()
        self.event.record(stream)

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)


class RcclCommunicator:
    def __init__(self, rank: int, world_size: int, broadcast_object=None):
        """``broadcast_object(obj) -> obj`` (rank 0's value on every rank) bootstraps the unique id when
        ``world_size > 1``; the calling process must already be bound to its GPU (``torch.cuda.set_device``)."""
        from ..ops._ext import require
        C = require()
        C.rccl_load(torch_rccl_path())
        uid = C.rccl_unique_id() if rank == 0 else None
        if world_size > 1:
            assert broadcast_object is not None, "multi-rank RCCL bootstrap needs an object broadcast"
            uid = broadcast_object(uid)
        self.rank, self.world_size = rank, world_size
        self.version = int(C.rccl_version())
        self._comm = C.RcclComm(uid, world_size, rank)

    @property
    def device(self) -> int:
        return int(self._comm.device)

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> EventWork:
        """In place on the current stream; returns its completion handle."""
        self._comm.all_reduce_(t, op)
        return EventWork()

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> EventWork:
        self._comm.broadcast_(t, root)
        return EventWork()

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> EventWork:
        self._comm.all_gather(out, inp)
        return EventWork()

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum") -> EventWork:
        self._comm.reduce_scatter(out, inp, op)
        return EventWork()

    def close(self):
        """Destroy the communicator (waits for its outstanding collectives)."""
        if self._comm is not None:
            self._comm = None   # the C++ destructor calls ncclCommDestroy

    def abort(self):
        """Failure path: tear down without waiting for peers."""
        if self._comm is not None:
            self._comm.abort()
            self._comm = None
