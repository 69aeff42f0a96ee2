"""HIP-graph replay of the fused training step (the MI355X answer to a tracing compiler: the executor's ~1000
kernel launches per step are recorded once and replayed as one graph launch).

``GraphedStep(eng, opt)`` captures ``eng.forward_backward(xs, labels)`` — both pathway streams, the weight-gradient
side streams and their joins become graph dependencies — plus, optionally, the fused SGD + bf16 re-pack kernels
(``FusedSGD.graph_kernels``), into one ``torch.cuda.CUDAGraph`` per (input buffers, accumulate, optimizer) key.
What stays outside the graph, per replay: the labels copy into the static label buffer and the lr refresh
(``FusedSGD.set_lr_tensor``).  The dropout key advances on the device (``FusedNet._head_forward``), so every replay
draws a fresh mask.  Inputs must be the same tensors (addresses) at every replay of a key: the double-buffered
preprocessing of ``bench.py`` yields two keys.

Valid after the autotuning step (no tuning launches, every workspace already allocated) and only for one
process per job without a gradient hook (the bucketed RCCL all-reduce runs eagerly; graphs are a launch-overhead
tool for the single-GPU / small-batch regime — the reference recipe's per-GPU batch is 8, run_slowfast_r50.sh).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch


class GraphedStep:
    def __init__(self, eng, opt=None):
        assert eng.grad_hook is None, "graph capture runs without the DDP gradient hook (single process)"
        assert eng._ms_warm, "capture after the first (autotuning) training step"
        self.eng, self.opt = eng, opt
        self.graphs: Dict[Tuple, Tuple[torch.cuda.CUDAGraph, torch.Tensor, torch.Tensor]] = {}
        self.labels: Optional[torch.Tensor] = None
        self.pool = None   # one private memory pool shared by every captured key

    def __call__(self, xs: List, labels: torch.Tensor, loss_scale: float = 1.0, accumulate: bool = False,
                 optimizer_step: bool = True):
        """One replayed micro-step; returns (loss [device scalar], logits) — graph-owned outputs, overwritten by
        the next replay of the same key."""
        eng = self.eng
        if self.labels is None or self.labels.shape != labels.shape or self.labels.dtype != labels.dtype:
            # graphs captured earlier read the old label buffer: they are invalid once it is replaced
            self.labels = torch.empty_like(labels, device=eng.device)
            self.graphs.clear()
        self.labels.copy_(labels, non_blocking=True)
        step = optimizer_step and self.opt is not None
        if step:
            self.opt.set_lr_tensor()
        key = (tuple(x.t.data_ptr() for x in xs), self.labels.data_ptr(), bool(accumulate), step, float(loss_scale))
        entry = self.graphs.get(key)
        if entry is None:
            entry = self._capture(xs, loss_scale, accumulate, step)
            self.graphs[key] = entry
        g, loss, logits = entry
        eng.flat.zeroed = False
        g.replay()
        return loss[0], logits

    def _capture(self, xs, loss_scale, accumulate, step):
        eng = self.eng
        torch.cuda.synchronize(eng.device)
        g = torch.cuda.CUDAGraph()
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        with torch.cuda.graph(g, pool=self.pool):
            loss, logits = eng.forward_backward(xs, self.labels, loss_scale=loss_scale, accumulate=accumulate)
            if step:
                self.opt.graph_kernels()
            out_loss = loss.reshape(1)
        torch.cuda.synchronize(eng.device)
        return g, out_loss, logits
