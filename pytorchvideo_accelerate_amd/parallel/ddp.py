"""Bucketed gradient all-reduce over RCCL, overlapped with the backward pass.

The flat fp32 gradient buffer (``models/fused.FlatParams``) is laid out in reverse execution order, so
the backward pass finalises it front to back.  ``GradSync`` cuts it into contiguous buckets; whenever
the executor reports that everything below offset ``x`` is final (``progress(x)``), every bucket that
ends at or below ``x`` is all-reduced immediately with ``async_op=True``.  ProcessGroupNCCL enqueues the
collective on its own (high-priority, see ``dist.DistState.from_env``) stream *after* the work already
queued on the compute stream, so bucket k's RCCL ring runs concurrently with the dgrad/wgrad kernels of
the remaining layers; ``finish()`` makes the compute stream wait for the outstanding collectives before
the optimizer step.

Differences to ``torch.nn.parallel.DistributedDataParallel`` as the reference uses it (SURVEY.md D4/C4,
reference ``run.py:196-198,257``), all math-identical:
* no per-parameter autograd hooks and no bucket copies (gradients *are* the buckets — the analogue of
  ``gradient_as_bucket_view=True``), averaging via ``ReduceOp.AVG`` inside RCCL;
* ``sync=False`` micro-steps under gradient accumulation skip the all-reduce (``no_sync``) — the
  reference all-reduces every micro-step;
* bucket size defaults to 32 MiB: large enough that each ring step is bandwidth- not latency-bound on
  a single xGMI link (≈153 GB/s), small enough to give ≥4 buckets for SlowFast-R50's 135 MiB.  Like
  DDP's ``_DEFAULT_FIRST_BUCKET_BYTES`` the first bucket is small (``first_mb``) so communication starts
  as soon as the head and the last residual unit are done.

Framework-owned communication stream: the bucket's gradients are produced on several HIP streams (the
slow-pathway stream, the fast-pathway stream and their weight-gradient streams).  ``producers`` (set by the executor)
lists them; at each bucket launch an event is recorded on every producer and the comm stream waits on all of them
before the collective is issued from it, so no compute stream ever waits for another one (or for the network) before
``finish()`` — buckets can be reported per residual block even while both pathways and their weight-gradient streams
are in flight.  Without ``producers`` (or for CPU gradients) the collective follows the current stream.

``PVA_COMM=rccl`` (``dist.DistState.comm``): the collective is the framework's own RCCL communicator's
``ncclAllReduce(avg)`` enqueued on that comm stream (``parallel/rccl.py``) instead of ProcessGroupNCCL's.

Options beyond DDP's defaults: ``grad_dtype=torch.bfloat16`` all-reduces a bf16 copy of each bucket
(half the xGMI bytes; the analogue of DDP's ``bf16_compress_hook``) and ``timing=True`` records, per
step, every bucket's ready→reduced latency and the *exposed* communication time (how long the compute
stream waited in ``finish()``), exported by :meth:`stats`.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import torch

from ..utils.profiling import trace_mark, trace_range
from .dist import DistState


class GradSync:
    def __init__(self, grad: torch.Tensor, state: DistState, bucket_mb: float = 32.0,
                 boundaries: Optional[List[int]] = None, first_mb: Optional[float] = None,
                 grad_dtype: Optional[torch.dtype] = None, timing: bool = False):
        self.grad = grad
        self.state = state
        self.enabled = state.multi
        n = grad.numel()
        cap = max(1, int(bucket_mb * (1 << 20) / grad.element_size()))
        first = cap if first_mb is None else max(1, int(first_mb * (1 << 20) / grad.element_size()))
        # cut at the given parameter boundaries (so a bucket never splits a tensor) near the cap
        cuts = [0]
        if boundaries:
            last = 0
            for b in boundaries:
                if b - last >= (first if len(cuts) == 1 else cap):
                    cuts.append(b)
                    last = b
        else:
            if first < n:
                cuts.append(first)
            cuts += list(range(cuts[-1] + cap, n, cap))
        if cuts[-1] != n:
            cuts.append(n)
        self.buckets: List[Tuple[int, int]] = [(cuts[i], cuts[i + 1]) for i in range(len(cuts) - 1)]
        self.grad_dtype = grad_dtype if grad_dtype not in (None, grad.dtype) else None
        self._lowp: Optional[torch.Tensor] = None
        # per-bucket timing needs a non-blocking Work.wait (RCCL: a stream wait); with gloo it would block the host
        # inside backward and serialise every bucket, so the gloo rehearsal runs untimed
        self.timing = timing and grad.is_cuda and state.backend == "nccl"
        self._comm_stream = torch.cuda.Stream(grad.device) if self.timing else None
        # the framework's own communication stream and the executor's gradient-producing streams (GPU gradients:
        # RCCL, and the gloo rehearsal of the same schedule on one GPU, whose CUDA work follows the issuing stream)
        self.producers: Optional[Callable[[], List]] = None
        self._cstream = torch.cuda.Stream(grad.device, priority=-1) if (self.enabled and grad.is_cuda) else None
        self._ev: List = []          # per step: (list of (ready, done) per bucket, (exp0, exp1))
        self._next = 0
        self._works = []
        self._bev = []
        self.active = False

    def restrict(self, lo: int, hi: int):
        """Only all-reduce grad[lo:hi] (e.g. frozen backbone: just the head)."""
        self.buckets = [(max(a, lo), min(b, hi)) for a, b in self.buckets if a < hi and b > lo]

    def begin(self, sync: bool = True):
        """Start a backward pass; ``sync=False`` = no_sync micro-step (accumulate locally)."""
        self._next = 0
        self._works = []
        self._bev = []
        self.active = self.enabled and sync

    def _event(self, stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    @property
    def multi_stream(self) -> bool:
        """Whether bucket launches wait on every producing stream themselves (executor: report per block, no joins)."""
        return self._cstream is not None and self.producers is not None

    def _launch(self, b: int):
        import torch.distributed as dist
        lo, hi = self.buckets[b]
        t = self.grad[lo:hi]
        cs = self._cstream if self.multi_stream else None
        if cs is not None:   # the comm stream joins every producer at this point (events, no compute-stream wait)
            for st in self.producers():
                cs.wait_event(self._event(st))
        ctx = torch.cuda.stream(cs) if cs is not None else None
        if ctx is not None:
            ctx.__enter__()
        try:
            ready = self._event() if self.timing else None
            if self.grad_dtype is not None:
                if self._lowp is None:
                    self._lowp = torch.empty(self.grad.numel(), dtype=self.grad_dtype, device=self.grad.device)
                low = self._lowp[lo:hi]
                low.copy_(t)
                comm = low
            else:
                comm = t
            with trace_range(f"allreduce/bucket{b}"):
                if self.state.comm is not None:   # framework-owned communicator: ncclAllReduce on this stream
                    w = self.state.comm.all_reduce_(comm, "avg")
                    post = None
                elif self.state.backend == "nccl":
                    w = dist.all_reduce(comm, op=dist.ReduceOp.AVG, async_op=True)
                    post = None
                else:
                    w = dist.all_reduce(comm, op=dist.ReduceOp.SUM, async_op=True)
                    post = "div"
        finally:
            if ctx is not None:
                ctx.__exit__(None, None, None)
        self._works.append((w, t, comm, post))
        if self.timing:
            # the side stream waits for this collective only: its event marks the bucket's completion
            with torch.cuda.stream(self._comm_stream):
                w.wait()
                done = self._event()
            self._bev.append((ready, done))

    def progress(self, offset: int):
        """Everything in grad[:offset] is final."""
        if not self.active:
            return
        while self._next < len(self.buckets) and self.buckets[self._next][1] <= offset:
            self._launch(self._next)
            self._next += 1

    def finish(self):
        if not self.active:
            return
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        e0 = self._event() if self.timing else None
        for b, (w, t, comm, post) in enumerate(self._works):
            trace_mark(f"allreduce/wait{b}")
            w.wait()   # the CURRENT (compute) stream waits for the collective
            if post == "div":
                comm.div_(self.state.world_size)
            if comm is not t:
                t.copy_(comm)
        if self.timing:
            self._ev.append((self._bev, (e0, self._event())))
        self._works = []
        self._bev = []
        self.active = False

    def stats(self, reset: bool = True) -> Dict[str, float]:
        """Mean per step over the recorded steps (synchronizes): ``comm_exposed_ms`` (compute stream
        blocked on communication), ``comm_bucket_ms`` (sum of bucket ready→reduced latencies),
        ``comm_last_bucket_ms``.  Empty when timing is off or nothing was synchronised."""
        if not self._ev:
            return {}
        torch.cuda.synchronize()
        n = len(self._ev)
        exposed = sum(a.elapsed_time(b) for _, (a, b) in self._ev) / n
        bucket = sum(sum(r.elapsed_time(d) for r, d in bev) for bev, _ in self._ev) / n
        last = sum((bev[-1][0].elapsed_time(bev[-1][1]) if bev else 0.0) for bev, _ in self._ev) / n
        if reset:
            self._ev = []
        return {"comm_exposed_ms": round(exposed, 3), "comm_bucket_ms": round(bucket, 3),
                "comm_last_bucket_ms": round(last, 3), "buckets": len(self.buckets)}
