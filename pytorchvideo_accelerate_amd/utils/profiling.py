"""Step-phase timers for the training loop (SURVEY.md §5 tracing / profiling).

:class:`StepTimer` records per-step phases — ``data`` (host wait for the next batch), ``fwd_bwd`` (forward +
backward + gradient-bucket launch), ``comm`` (wait for the last RCCL all-reduce), ``opt`` (fused SGD +
weight re-pack) — with HIP events on GPU (no synchronisation inside the step; resolved lazily at
``summary()``) and ``perf_counter`` on CPU.  ``summary()`` returns p50/p90 step time, clips/s and mean
phase times, logged by the trainer as ``step_time_ms``, ``step_time_p90_ms``, ``clips_per_sec``,
``data_wait_ms``, ``fwd_bwd_ms``, ``comm_ms``, ``opt_ms``.

For kernel-level traces use ``rocprofv3 --kernel-trace --stats`` (scripts/gpu_bench.sh PROFILE=...) or the
per-op event profiler of the fused executor (``FusedNet.prof`` / scripts/layer_profile.py).

ROCTx ranges (:func:`trace_range`, :func:`trace_mark`) name the host-side phases on the rocprofv3 timeline
(``rocprofv3 --marker-trace --kernel-trace``): ``fwd/b{i}`` / ``bwd/b{i}`` per stage, ``allreduce/bucket{k}``
per gradient bucket, ``step`` / ``sgd`` in the trainer and bench.  They call libroctx through the in-tree
extension and cost ~1 µs each; without a profiler attached they are no-ops.  ``PVA_ROCTX=0`` disables them.
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Dict, List, Optional

import torch

_RTX = None   # extension module with range_push/range_pop/trace_mark, False when unavailable


def _rtx():
    global _RTX
    if _RTX is None:
        _RTX = False
        if os.environ.get("PVA_ROCTX", "1") != "0" and torch.cuda.is_available():
            from ..ops._ext import load
            mod = load()
            if mod is not None and hasattr(mod, "range_push"):
                _RTX = mod
    return _RTX


@contextlib.contextmanager
def trace_range(name: str):
    """ROCTx push/pop range around the block (host timeline)."""
    m = _rtx()
    if not m:
        yield
        return
    m.range_push(name)
    try:
        yield
    finally:
        m.range_pop()


def trace_mark(name: str):
    """ROCTx instantaneous marker."""
    m = _rtx()
    if m:
        m.trace_mark(name)


class StepTimer:
    PHASES = ("data", "fwd_bwd", "comm", "opt")

    def __init__(self, device: torch.device, window: int = 200):
        self.gpu = torch.device(device).type == "cuda"
        self.window = window
        self._pending: List[Dict] = []   # steps with unresolved events
        self.steps: List[Dict[str, float]] = []
        self._cur: Optional[Dict] = None

    def begin_step(self):
        self._cur = {"t0": time.perf_counter(), "ev": {}, "host": {}}

    @contextlib.contextmanager
    def host(self, name: str):
        """Host-side wall time (e.g. waiting for the data loader)."""
        t = time.perf_counter()
        yield
        if self._cur is not None:
            self._cur["host"][name] = self._cur["host"].get(name, 0.0) + (time.perf_counter() - t) * 1e3

    @contextlib.contextmanager
    def phase(self, name: str):
        """Device time of the work enqueued inside the block (wall time on CPU)."""
        if self._cur is None:
            yield
            return
        if self.gpu:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            yield
            e1.record()
            self._cur["ev"].setdefault(name, []).append((e0, e1))
        else:
            t = time.perf_counter()
            yield
            self._cur["host"][name] = self._cur["host"].get(name, 0.0) + (time.perf_counter() - t) * 1e3

    def end_step(self, clips: int):
        if self._cur is None:
            return
        c = self._cur
        c["clips"] = clips
        if self.gpu:
            c["end"] = torch.cuda.Event(enable_timing=True)
            c["end"].record()
        c["wall"] = (time.perf_counter() - c["t0"]) * 1e3
        self._pending.append(c)
        self._cur = None

    def _resolve(self):
        if not self._pending:
            return
        if self.gpu:
            torch.cuda.synchronize()
        for c in self._pending:
            rec = dict(c["host"])
            for name, evs in c["ev"].items():
                rec[name] = rec.get(name, 0.0) + sum(a.elapsed_time(b) for a, b in evs)
            rec["clips"] = c["clips"]
            rec["wall"] = c["wall"]
            self.steps.append(rec)
        self._pending.clear()
        self.steps = self.steps[-self.window:]

    def summary(self, skip_first: int = 0) -> Dict[str, float]:
        self._resolve()
        st = self.steps[skip_first:] or self.steps
        if not st:
            return {}
        walls = sorted(s["wall"] for s in st)
        q = lambda p: walls[min(len(walls) - 1, int(p * len(walls)))]
        out = {"step_time_ms": q(0.5), "step_time_p90_ms": q(0.9),
               "clips_per_sec": sum(s["clips"] for s in st) / max(sum(walls) / 1e3, 1e-9)}
        for ph in self.PHASES:
            vals = [s.get(ph, 0.0) for s in st]
            out[f"{'data_wait' if ph == 'data' else ph}_ms"] = sum(vals) / len(vals)
        return out
