"""Fused SGD(+momentum, +weight decay) over the flat fp32 master buffer.

``FusedSGD`` *is a* ``torch.optim.SGD`` (so ``CosineAnnealingLR``, ``state_dict``/``load_state_dict`` and
accelerate-format checkpoints behave exactly like the reference's optimizer, ``run.py:192``), but its
``step`` is ONE kernel launch over every parameter (``sgd_momentum_kernel``) followed by ONE
multi-tensor bf16 weight-pack launch, instead of PyTorch's per-tensor foreach chain.
Momentum buffers are views into one flat fp32 buffer so they checkpoint as ordinary per-parameter
``momentum_buffer`` entries.  The learning rate is read on device from a 1-element tensor so a captured
HIP graph replays with the live schedule.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ._ext import require


class FusedSGD(torch.optim.SGD):
    def __init__(self, flat, lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 1e-4,
                 after_step: Optional[Callable[[], None]] = None, params=None):
        # ``params`` defaults to the flat buffer's parameter list; reference order can be passed so that
        # state_dict indices match ``model.parameters()`` (what torch.optim.SGD(model.parameters()) saves).
        super().__init__(params if params is not None else flat.params, lr=lr, momentum=momentum,
                         weight_decay=weight_decay)
        self.flat = flat
        self.after_step = after_step
        self.buf = torch.zeros_like(flat.data)
        self.lr_t = torch.full((1,), float(lr), device=flat.data.device, dtype=torch.float32)
        self.found_inf = torch.zeros(1, device=flat.data.device, dtype=torch.int32)
        self._first = True
        self._C = require() if flat.data.is_cuda else None
        self.span = None            # (lo, hi): only this slice of the flat buffer trains (frozen backbone)
        self.step_was_skipped = False

    def _bind_state(self):
        for p in self.flat.params:
            st = self.state[p]
            a, b = self.flat.span(p)
            st["momentum_buffer"] = self.buf[a:b].view(p.shape)

    def set_lr_tensor(self):
        self.lr_t.fill_(float(self.param_groups[0]["lr"]))

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0, check_finite: bool = False):
        """One SGD step on ``grad * grad_scale``.  ``check_finite`` (fp16 loss scaling): a non-finite
        gradient turns the whole step into a no-op (parameters and momentum untouched) and sets
        ``step_was_skipped`` (one device->host read of the flag)."""
        g = self.param_groups[0]
        lo, hi = self.span if self.span is not None else (0, self.flat.numel)
        data, grad, buf = self.flat.data[lo:hi], self.flat.grad[lo:hi], self.buf[lo:hi]
        skipped = False
        if self._C is None:  # CPU path: plain torch math on the flat buffers
            lr, m, wd = g["lr"], g["momentum"], g["weight_decay"]
            if check_finite and not bool(torch.isfinite(grad * grad_scale).all()):
                skipped = True
            else:
                d = grad * grad_scale + wd * data
                if self._first:
                    buf.copy_(d)
                else:
                    buf.mul_(m).add_(d)
                data.add_(buf, alpha=-lr)
        else:
            self.set_lr_tensor()
            if check_finite:
                self.found_inf.zero_()
                self._C.nonfinite_check(grad, grad_scale, self.found_inf)
                self._C.sgd_momentum(data, grad, buf, self.lr_t, g["momentum"], g["weight_decay"], grad_scale,
                                     1 if self._first else 0, None, self.found_inf)
                skipped = bool(self.found_inf.item())
            else:
                self._C.sgd_momentum(data, grad, buf, self.lr_t, g["momentum"],
                                     g["weight_decay"], grad_scale, 1 if self._first else 0, None)
        self.step_was_skipped = skipped
        if skipped:
            return None
        if self._first:
            self._bind_state()
            self._first = False
        if self.after_step is not None:
            self.after_step()
        return None

    def graph_kernels(self):
        """The device work of one plain (non-first, no loss-scale check) step, for capture into a HIP graph:
        the lr lives in ``lr_t`` (refreshed by ``set_lr_tensor`` before each replay, outside the graph)."""
        assert self._C is not None and not self._first, "capture after the first (state-binding) step"
        g = self.param_groups[0]
        lo, hi = self.span if self.span is not None else (0, self.flat.numel)
        self._C.sgd_momentum(self.flat.data[lo:hi], self.flat.grad[lo:hi], self.buf[lo:hi], self.lr_t,
                             g["momentum"], g["weight_decay"], 1.0, 0, None)
        if self.after_step is not None:
            self.after_step()

    def zero_grad(self, set_to_none: bool = True):
        # No memset: the next backward *overwrites* the flat gradient buffer instead of accumulating
        # (wgrad/BN kernels take beta = 0; FusedNet.forward_backward reads ``flat.zeroed``).
        self.flat.zeroed = True

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        any_buf = False
        for p in self.flat.params:
            st = self.state.get(p, {})
            mb = st.get("momentum_buffer")
            if mb is not None:
                a, b = self.flat.span(p)
                self.buf[a:b].copy_(mb.reshape(-1))
                any_buf = True
        if any_buf:
            self._bind_state()
            self._first = False


class FusedGradScaler:
    """Dynamic loss scaling for ``--mixed_precision fp16`` on the fused path (reference recipe,
    ``run_slowfast_r50.sh:7``; accelerate/torch ``GradScaler`` semantics):

    * the backward pass computes gradients of ``loss * scale`` (the executor folds ``scale`` into the
      head's dlogits, so no extra pass);
    * ``step(optimizer)`` unscales inside the fused SGD kernel (``grad_scale = 1/scale``) after a
      device-side non-finite check; an overflowing step is skipped entirely (``optimizer.step_was_skipped``,
      which also skips the LR scheduler step, accelerate ``scheduler.py:66-68``);
    * ``update()``: ×``backoff_factor`` after an overflow, ×``growth_factor`` after ``growth_interval``
      consecutive clean steps (torch defaults 2**16, 2.0, 0.5, 2000).

    ``state_dict`` has torch ``GradScaler``'s keys, so ``scaler.pt`` checkpoints interoperate.
    Compute stays bf16 (MFMA) with fp32 master weights — the loss-scale state machine is what fp16
    training semantics need; bf16 needs no scaling for range, so overflow skips are rare."""

    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000, enabled: bool = True):
        self._scale = float(init_scale)
        self._growth_factor = float(growth_factor)
        self._backoff_factor = float(backoff_factor)
        self._growth_interval = int(growth_interval)
        self._growth_tracker = 0
        self._enabled = enabled
        self._found_inf = False

    def is_enabled(self) -> bool:
        return self._enabled

    def get_scale(self) -> float:
        return self._scale if self._enabled else 1.0

    def step(self, optimizer: FusedSGD):
        optimizer.step(grad_scale=1.0 / self.get_scale(), check_finite=self._enabled)
        self._found_inf = bool(optimizer.step_was_skipped)

    def update(self):
        if not self._enabled:
            return
        if self._found_inf:
            self._scale *= self._backoff_factor
            self._growth_tracker = 0
        else:
            self._growth_tracker += 1
            if self._growth_tracker == self._growth_interval:
                self._scale *= self._growth_factor
                self._growth_tracker = 0

    def state_dict(self):
        return {"scale": self._scale, "growth_factor": self._growth_factor, "backoff_factor": self._backoff_factor,
                "growth_interval": self._growth_interval, "_growth_tracker": self._growth_tracker}

    def load_state_dict(self, sd):
        self._scale = float(sd["scale"])
        self._growth_factor = float(sd.get("growth_factor", self._growth_factor))
        self._backoff_factor = float(sd.get("backoff_factor", self._backoff_factor))
        self._growth_interval = int(sd.get("growth_interval", self._growth_interval))
        self._growth_tracker = int(sd.get("_growth_tracker", 0))
