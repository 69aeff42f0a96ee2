"""Main-process training progress bar (reference ``run.py:22,233,235,263,288``: ``tqdm`` over
``num_epochs * len(train_loader)`` steps, description ``"Epoch: %s"`` while training and ``"Val Epoch: %s"``
while evaluating, ``update(1)`` per micro-step, disabled off the main process).

Uses ``tqdm`` when importable; otherwise a small stderr fallback with the same interface, so the bar is
never a hard dependency (the reference imports tqdm without listing it in ``requirements.txt``).
"""
from __future__ import annotations

import sys
import time


class _FallbackBar:
    def __init__(self, total: int, disable: bool = False, file=None, mininterval: float = 1.0):
        self.total, self.n, self.disable = total, 0, disable
        self.desc, self.postfix = "", ""
        self.file = file or sys.stderr
        self.mininterval = mininterval
        self._t0 = time.perf_counter()
        self._last = 0.0

    def set_description_str(self, s: str):
        self.desc = s
        self._render(force=True)

    def set_postfix_str(self, s: str):
        self.postfix = s

    def update(self, n: int = 1):
        self.n += n
        self._render()

    def _render(self, force: bool = False):
        if self.disable:
            return
        now = time.perf_counter()
        if not force and now - self._last < self.mininterval and self.n < self.total:
            return
        self._last = now
        rate = self.n / max(now - self._t0, 1e-9)
        pct = 100.0 * self.n / max(self.total, 1)
        self.file.write(f"\r{self.desc}: {pct:3.0f}% {self.n}/{self.total} [{rate:.2f}it/s] {self.postfix}")
        self.file.flush()

    def close(self):
        if not self.disable:
            self._render(force=True)
            self.file.write("\n")
            self.file.flush()


def progress_bar(total: int, disable: bool = False, file=None):
    try:
        from tqdm.auto import tqdm
    except Exception:  # pragma: no cover - tqdm is optional
        return _FallbackBar(total, disable=disable, file=file)
    return tqdm(range(total), disable=disable, file=file)
