"""Experiment trackers (accelerate ``log_with="all"``, SURVEY.md D12 / §5 metrics).

``log_with="all"`` selects every tracker whose library imports: a JSON-lines tracker (always available,
``<logging_dir>/<run>/metrics.jsonl``), TensorBoard (``torch.utils.tensorboard`` when the
``tensorboard`` package is present) and Weights & Biases (when ``wandb`` imports; offline here).
All methods are no-ops off the main process, like accelerate.
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, List, Optional


class JsonlTracker:
    name = "jsonl"

    def __init__(self, run_name: str, logging_dir: str):
        self.dir = os.path.join(logging_dir, run_name)
        os.makedirs(self.dir, exist_ok=True)
        self.path = os.path.join(self.dir, "metrics.jsonl")
        self._fh = open(self.path, "a")

    def store_init_configuration(self, config: Dict[str, Any]):
        with open(os.path.join(self.dir, "config.json"), "w") as fh:
            json.dump({k: (v if isinstance(v, (int, float, str, bool, type(None), list)) else str(v))
                       for k, v in config.items()}, fh, indent=1)

    def log(self, values: Dict[str, Any], step: Optional[int] = None):
        rec = {"step": step, "time": time.time()}
        for k, v in values.items():
            rec[k] = float(v) if hasattr(v, "__float__") and not isinstance(v, (int, str)) else v
        self._fh.write(json.dumps(rec) + "\n")
        self._fh.flush()

    def finish(self):
        self._fh.close()


class TensorBoardTracker:
    name = "tensorboard"

    def __init__(self, run_name: str, logging_dir: str):
        from torch.utils.tensorboard import SummaryWriter  # needs the tensorboard package
        self.writer = SummaryWriter(os.path.join(logging_dir, run_name))

    def store_init_configuration(self, config):
        self.writer.add_text("config", json.dumps({k: str(v) for k, v in config.items()}))

    def log(self, values, step=None):
        for k, v in values.items():
            if isinstance(v, (int, float)):
                self.writer.add_scalar(k, v, global_step=step)
        self.writer.flush()

    def finish(self):
        self.writer.close()


class WandBTracker:
    name = "wandb"

    def __init__(self, run_name: str, logging_dir: str):
        import wandb
        os.environ.setdefault("WANDB_MODE", "offline")
        self.run = wandb.init(project=run_name, dir=logging_dir)

    def store_init_configuration(self, config):
        self.run.config.update(config, allow_val_change=True)

    def log(self, values, step=None):
        self.run.log(values, step=step)

    def finish(self):
        self.run.finish()


_AVAILABLE = {"jsonl": JsonlTracker, "tensorboard": TensorBoardTracker, "wandb": WandBTracker}


def _importable(name: str) -> bool:
    try:
        if name == "tensorboard":
            import tensorboard  # noqa: F401
        elif name == "wandb":
            import wandb  # noqa: F401
        return True
    except Exception:
        return False


class Trackers:
    def __init__(self, log_with="all", logging_dir: str = "runs", is_main: bool = True):
        self.is_main = is_main
        self.logging_dir = logging_dir
        if log_with in (None, "none"):
            self.names: List[str] = []
        elif log_with == "all":
            self.names = [n for n in _AVAILABLE if _importable(n)]
        else:
            self.names = [log_with] if isinstance(log_with, str) else list(log_with)
        self.trackers = []

    def init(self, run_name: str, config: Optional[Dict[str, Any]] = None):
        if not self.is_main:
            return
        for n in self.names:
            try:
                t = _AVAILABLE[n](run_name, self.logging_dir)
            except Exception:
                continue
            if config is not None:
                t.store_init_configuration(config)
            self.trackers.append(t)

    def log(self, values: Dict[str, Any], step: Optional[int] = None):
        if not self.is_main:
            return
        for t in self.trackers:
            t.log(values, step=step)

    def finish(self):
        if not self.is_main:
            return
        for t in self.trackers:
            t.finish()
        self.trackers = []
