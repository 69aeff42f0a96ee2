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
    def step(self, closure=None, grad_scale: float = 1.0):
        g = self.param_groups[0]
        lo, hi = self.span if self.span is not None else (0, self.flat.numel)
        data, grad, buf = self.flat.data[lo:hi], self.flat.grad[lo:hi], self.buf[lo:hi]
        if self._C is None:  # CPU path: plain torch math on the flat buffers
            lr, m, wd = g["lr"], g["momentum"], g["weight_decay"]
            d = grad * grad_scale + wd * data
            if self._first:
                buf.copy_(d)
            else:
                buf.mul_(m).add_(d)
            data.add_(buf, alpha=-lr)
        else:
            self.set_lr_tensor()
            self._C.sgd_momentum(data, grad, buf, self.lr_t, g["momentum"],
                                 g["weight_decay"], grad_scale, 1 if self._first else 0, None)
        if self._first:
            self._bind_state()
            self._first = False
        if self.after_step is not None:
            self.after_step()
        return None

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
