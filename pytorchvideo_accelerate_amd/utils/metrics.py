"""Multiclass top-1 accuracy with distributed sync (torchmetrics ``Accuracy`` as the reference uses it,
SURVEY.md D23 / C6-C7).

``update``/``forward`` accumulate (correct, total) counters on the device; ``compute`` all-reduces the two
int64 counters once across ranks (the reference all-gathers predictions and labels every eval step and
again in ``compute``: same result, one collective per epoch instead of 2 per step + 1)."""
from __future__ import annotations

from typing import Optional

import torch


class Accuracy:
    def __init__(self, device=None, state=None):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.state = state  # parallel.dist.DistState (optional)
        self.reset()

    def reset(self):
        self.correct = torch.zeros((), dtype=torch.long, device=self.device)
        self.total = torch.zeros((), dtype=torch.long, device=self.device)

    @staticmethod
    def _preds(x: torch.Tensor) -> torch.Tensor:
        return x.argmax(-1) if x.is_floating_point() and x.dim() > 1 else x

    def update(self, preds: torch.Tensor, target: torch.Tensor):
        p = self._preds(preds).to(self.device)
        t = target.to(self.device)
        self.correct += (p == t).sum()
        self.total += t.numel()

    def update_counts(self, counts: torch.Tensor):
        """Add device-side (correct, total) int64 counters (e.g. from the fused head's argmax kernel)."""
        c = counts.to(self.device)
        self.correct += c[0]
        self.total += c[1]

    def forward(self, preds: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        """Update and return this batch's (local) accuracy, like ``torchmetrics.Metric.forward``."""
        p = self._preds(preds).to(self.device)
        t = target.to(self.device)
        c = (p == t).sum()
        self.correct += c
        self.total += t.numel()
        return c.float() / max(t.numel(), 1)

    __call__ = forward

    def compute(self) -> torch.Tensor:
        c, n = self.correct.clone(), self.total.clone()
        if self.state is not None and getattr(self.state, "world_size", 1) > 1:
            self.state.all_reduce_(c, "sum")
            self.state.all_reduce_(n, "sum")
        return c.float() / n.clamp_min(1).float()
