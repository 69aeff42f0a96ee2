"""Execution back-ends behind one training-step interface.

* :class:`FusedBackend` — the MI355X path: ``models/fused.FusedNet`` (gfx950 kernels, bf16 or fp16) with the
  bucketed RCCL gradient all-reduce of ``parallel/ddp.GradSync`` overlapped with the backward pass.
* :class:`NativeF32Backend` — the reference default precision (``--mixed_precision no``) on the gfx950 fp32 kernels
  (``models/native32.NativeF32Net``: split-bf16 (bf16x6) MFMA convolutions, fp32 BatchNorm/pool/head), same bucketed all-reduce.
* :class:`TorchBackend` — the reference PyTorch modules with autograd: CPU runs (``--cpu``, gloo DDP), or
  autocast fp16/bf16 / fp32 modules on GPU when asked for (``--kernels torch``); its bucketed all-reduce overlaps backward through
  per-parameter gradient hooks, as DDP's reducer does.  Gradients land in the same flat buffer
  (``FlatParams``), so the optimizer, gradient sync and checkpointing code are shared.

Both expose ``train_step(batch, labels, loss_scale, sync) -> (loss, logits)``, ``eval_step``,
``flat`` and ``model`` (the pytorchvideo-keyed ``nn.Module`` used for ``state_dict``).
"""
from __future__ import annotations

import contextlib
from typing import List, Optional

import torch
import torch.nn.functional as F

from ..models.fused import FlatParams
from ..parallel.ddp import GradSync
from ..parallel.dist import DistState


def _ordered_params(model):
    return [(n, p) for n, p in reversed(list(model.named_parameters()))]


class TorchBackend:
    name = "torch"

    def __init__(self, model: torch.nn.Module, state: DistState, mixed_precision: str = "no",
                 bucket_mb: float = 32.0, trainable: Optional[List[torch.nn.Parameter]] = None):
        self.model = model.to(state.device)
        self.state = state
        self.device = state.device
        self.flat = FlatParams(_ordered_params(self.model), self.device)
        self.sync = GradSync(self.flat.grad, state, bucket_mb)
        self.mp = mixed_precision
        self.amp_dtype = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(mixed_precision)
        self.scaler = None
        self.timer = None
        if mixed_precision == "fp16" and self.device.type == "cuda":
            self.scaler = torch.amp.GradScaler("cuda")
        self._install_overlap()

    def _install_overlap(self):
        """DDP-style overlap of the gradient all-reduce with autograd (reference run.py:196-198,257 via DDP's
        reducer): a post-accumulate hook per parameter marks its gradient final; as soon as every parameter below a
        flat offset is final (the flat buffer is in reverse execution order), ``GradSync.progress`` launches the
        buckets that end there while backward continues.  Frozen parameters never get a gradient: they count as
        final from the start."""
        ps = self.flat.params
        self._ends = [self.flat.span(p)[1] for p in ps]
        self._frozen = [not p.requires_grad for p in ps]
        self._ready = list(self._frozen)
        self._front = 0
        for i, p in enumerate(ps):
            if p.requires_grad:
                p.register_post_accumulate_grad_hook(lambda _p, i=i: self._on_grad(i))

    def _on_grad(self, i: int):
        if not self.sync.active:
            return
        self._ready[i] = True
        f = self._front
        while f < len(self._ready) and self._ready[f]:
            f += 1
        if f != self._front:
            self._front = f
            self.sync.progress(self._ends[f - 1])

    def _autocast(self):
        if self.amp_dtype is None:
            return contextlib.nullcontext()
        return torch.autocast(self.device.type, dtype=self.amp_dtype)

    def _input(self, video):
        if isinstance(video, (list, tuple)):
            return [v.to(self.device, non_blocking=True) for v in video]
        return video.to(self.device, non_blocking=True)

    def train(self):
        self.model.train()

    def eval(self):
        self.model.eval()

    def train_step(self, video, labels, loss_scale: float = 1.0, sync: bool = True):
        if self.flat.zeroed:
            self.flat.grad.zero_()
            self.flat.zeroed = False
        x = self._input(video)
        labels = labels.to(self.device)
        with self._autocast():
            out = self.model(x)
        loss = F.cross_entropy(out.float(), labels)
        scaled = loss * loss_scale
        if self.scaler is not None:
            scaled = self.scaler.scale(scaled)
        self.flat.rebind()   # gradients accumulate in place into the flat buffer the buckets are cut from
        self.sync.begin(sync)
        self._ready = list(self._frozen)
        self._front = 0
        scaled.backward()     # buckets are all-reduced from the gradient hooks as backward finalises them
        self.flat.rebind()
        with (self.timer.phase("comm") if self.timer else contextlib.nullcontext()):
            self.sync.finish()
        return loss.detach(), out.detach().float()

    @torch.no_grad()
    def eval_step(self, video):
        with self._autocast():
            return self.model(self._input(video)).float()

    def after_optimizer_step(self):
        pass


class NativeF32Backend:
    """fp32 training on the native fp32 kernels (reference run.py:330 default ``mixed_precision="no"``)."""
    name = "native32"

    def __init__(self, model: torch.nn.Module, state: DistState, bucket_mb: float = 32.0):
        from ..models.native32 import NativeF32Net
        self.state = state
        self.device = state.device
        self.net = NativeF32Net(model, self.device)
        self.model = model
        self.flat = self.net.flat
        bounds = sorted(set(self.flat.span(p)[1] for p in self.flat.params))
        self.sync = GradSync(self.flat.grad, state, bucket_mb, boundaries=bounds)
        self.net.grad_hook = self.sync.progress if state.multi else None
        # one producing stream: buckets leave from the sync's comm stream after an event on it
        self.sync.producers = lambda: [torch.cuda.current_stream(self.device)]
        self.scaler = None
        self.timer = None

    def train(self):
        self.model.train()

    def eval(self):
        self.model.eval()

    def train_step(self, video, labels, loss_scale: float = 1.0, sync: bool = True):
        t = self.timer
        with (t.phase("fwd_bwd") if t else contextlib.nullcontext()):
            self.sync.begin(sync)
            loss, logits = self.net.forward_backward(video, labels, loss_scale)
        with (t.phase("comm") if t else contextlib.nullcontext()):
            self.sync.finish()
        return loss, logits

    @torch.no_grad()
    def eval_step(self, video):
        return self.net.forward_eval(video)

    def eval_counts(self, logits, labels):
        return self.net.eval_counts(logits, labels)

    def after_optimizer_step(self):
        pass

    def reload_weights(self):
        self.flat.rebind()


class FusedBackend:
    name = "fused"

    def __init__(self, model: torch.nn.Module, state: DistState, bucket_mb: float = 32.0,
                 mixed_precision: str = "bf16"):
        from ..models.fused import FusedNet
        from ..ops.optim import FusedGradScaler
        self.state = state
        self.device = state.device
        dp = state.multi
        cdt = torch.float16 if mixed_precision == "fp16" else torch.bfloat16
        self.net = FusedNet(model, self.device, load_tuning=not dp, compute_dtype=cdt)
        if dp:   # identical autotuner choices on every rank
            self.net.tuner.agree = state.agree_times
            ts = self.net.tune_store
            # rank 0's persistent table, broadcast once (then only geometries missing from it are tuned and agreed)
            doc = state.broadcast_object(ts.read() if (ts is not None and state.rank == 0) else None)
            if ts is not None:
                ts.restore(doc)
                ts.writer = state.rank == 0
        self.model = model
        self.flat = self.net.flat
        bounds = sorted(set(self.flat.span(p)[1] for p in self.flat.params))
        self.sync = GradSync(self.flat.grad, state, bucket_mb, boundaries=bounds)
        self.net.grad_hook = self.sync.progress if state.multi else None
        self.sync.producers = self.net.producer_streams   # RCCL: buckets issued from the sync's own comm stream
        self.net.grad_multi_stream = self.sync.multi_stream
        # fp16: fp16 kernels plus the dynamic loss-scale state machine (GradScaler semantics: fp16 has 5 exponent bits)
        self.scaler = FusedGradScaler() if mixed_precision == "fp16" else None
        self._training = True
        self.timer = None   # utils.profiling.StepTimer (optional)

    def train(self):
        self._training = True
        self.model.train()

    def eval(self):
        self._training = False
        self.model.eval()

    def train_step(self, video, labels, loss_scale: float = 1.0, sync: bool = True):
        t = self.timer
        with (t.phase("fwd_bwd") if t else contextlib.nullcontext()):
            self.sync.begin(sync)
            if self.scaler is not None:
                loss_scale = loss_scale * self.scaler.get_scale()
            loss, logits = self.net.forward_backward(video, labels.to(self.device), loss_scale)
        with (t.phase("comm") if t else contextlib.nullcontext()):
            self.sync.finish()
        return loss, logits

    @torch.no_grad()
    def eval_step(self, video):
        return self.net.forward_eval(video)

    def eval_counts(self, logits, labels):
        """(correct, total) of one eval batch on the HIP argmax/count kernel."""
        return self.net.eval_counts(logits, labels)

    def after_optimizer_step(self):
        self.net.pack()

    def reload_weights(self):
        """After parameters were overwritten (checkpoint load): re-point views and re-pack bf16."""
        self.flat.rebind()
        self.net.pack()
