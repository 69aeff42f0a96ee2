"""A small ``accelerate.Accelerator`` equivalent for this engine.

Keeps the call surface the reference script uses (``run.py:135-325``): ``device``, ``state
.distributed_type``, ``is_main_process``, ``print``, ``prepare``, ``gather``, ``save_state``/``load_state``,
``register_for_checkpointing``, ``init_trackers``/``log``/``end_training``, ``wait_for_everyone`` — but
``prepare(model)`` returns an execution back-end (fused HIP kernels on GPU, PyTorch on CPU), not a DDP
wrapper, and the optimizer/scheduler are built on the back-end's flat parameter buffer.

Launch contract: works under ``accelerate launch``, ``torchrun`` / ``python -m torch.distributed.run``
(reads RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*) or plain ``python``; honours ``ACCELERATE_MIXED_PRECISION``
when ``mixed_precision`` is not given.
"""
from __future__ import annotations

import math
import os
from typing import Any, List, Optional

import torch

from ..ckpt.state import load_state as _load_state
from ..ckpt.state import save_state as _save_state
from ..parallel.dist import DistState
from ..utils.tracking import Trackers


class GlobalRateScheduler:
    """accelerate ``AcceleratedScheduler`` semantics: each ``step()`` advances the wrapped scheduler
    ``num_processes`` times (T_max counts *global* batches) and is skipped when the optimizer step was
    skipped (fp16 overflow)."""

    def __init__(self, scheduler, optimizer, num_processes: int):
        self.scheduler, self.optimizer, self.num_processes = scheduler, optimizer, num_processes

    def step(self):
        if getattr(self.optimizer, "step_was_skipped", False):
            return
        for _ in range(self.num_processes):
            self.scheduler.step()

    def get_last_lr(self):
        return self.scheduler.get_last_lr()

    def state_dict(self):
        return self.scheduler.state_dict()

    def load_state_dict(self, sd):
        self.scheduler.load_state_dict(sd)


class Accelerator:
    def __init__(self, cpu: bool = False, mixed_precision: Optional[str] = None, log_with="all",
                 logging_dir: str = ".", kernels: str = "auto", bucket_mb: float = 32.0):
        if mixed_precision is None:
            mixed_precision = os.environ.get("ACCELERATE_MIXED_PRECISION", "no")
        cpu = cpu or os.environ.get("ACCELERATE_USE_CPU", "").lower() in ("1", "true", "yes")
        self.mixed_precision = mixed_precision
        self.state = DistState.from_env(cpu=cpu)
        self.device = self.state.device
        self.trackers = Trackers(log_with, logging_dir, self.state.is_main_process)
        self.logging_dir = logging_dir
        self.bucket_mb = bucket_mb
        # Precision policy (what runs is what was asked for; recorded as ``compute_dtype``):
        #  * bf16 / fp16 on a GPU -> the fused gfx950 kernels in that dtype (bf16 or fp16 MFMA operands and
        #    activations, fp32 accumulation, statistics, master weights and optimizer); fp16 also runs the dynamic
        #    loss-scale state machine of the reference recipe (run_slowfast_r50.sh, GradScaler semantics);
        #  * "no" (the reference default, fp32 math) on a GPU -> the native fp32 kernels (kernels="fp32":
        #    fp32 activations, split-bf16 MFMA convolutions (three pieces, six products: fp32 accuracy) with fp32 accumulation, fp32 BatchNorm / pooling / head);
        #  * CPU, or kernels="torch" -> the PyTorch module path (fp32, or autocast for bf16 / fp16).
        if kernels == "auto":
            if self.device.type == "cuda":
                kernels = "fused" if mixed_precision in ("bf16", "fp16") else "fp32"
            else:
                kernels = "torch"
        if kernels == "fp32" and self.device.type != "cuda":
            raise ValueError("--kernels fp32 runs the gfx950 fp32 kernels: it needs a GPU")
        if kernels == "fused":
            self.compute_dtype = "fp16" if mixed_precision == "fp16" else "bf16"
        elif kernels == "fp32":
            if mixed_precision not in ("no", None):
                raise ValueError(f"--kernels fp32 is the --mixed_precision no path (got {mixed_precision})")
            self.compute_dtype = "fp32"
        else:
            self.compute_dtype = {"bf16": "bf16-autocast", "fp16": "fp16-autocast"}.get(mixed_precision, "fp32")
        self.kernels = kernels
        self._models: List[Any] = []
        self._optimizers: List[Any] = []
        self._schedulers: List[Any] = []
        self._custom: List[Any] = []
        self.step = 0

    # ------------------------------------------------------------------ state
    @property
    def is_main_process(self) -> bool:
        return self.state.is_main_process

    @property
    def num_processes(self) -> int:
        return self.state.world_size

    @property
    def process_index(self) -> int:
        return self.state.rank

    @property
    def distributed_type(self) -> str:
        return self.state.distributed_type

    def print(self, *args, **kw):
        if self.is_main_process:
            print(*args, **kw, flush=True)

    def wait_for_everyone(self):
        self.state.barrier()

    # ------------------------------------------------------------------ prepare
    def prepare_model(self, model: torch.nn.Module):
        from .backends import FusedBackend, NativeF32Backend, TorchBackend
        if self.kernels == "fused":
            be = FusedBackend(model, self.state, self.bucket_mb, mixed_precision=self.mixed_precision)
        elif self.kernels == "fp32":
            be = NativeF32Backend(model, self.state, self.bucket_mb)
        else:
            be = TorchBackend(model, self.state, self.mixed_precision, self.bucket_mb)
        # rank-0 parameters + BN buffers everywhere (DDP construction broadcast)
        self.state.broadcast_tensors([be.flat.data] + list(model.buffers()))
        if hasattr(be, "reload_weights"):
            be.reload_weights()
        self._models.append(be)
        return be

    def make_optimizer(self, backend, lr: float, momentum: float, weight_decay: float):
        from ..ops.optim import FusedSGD
        params = list(backend.model.parameters())  # state_dict indices == torch.optim.SGD(model.parameters())
        opt = FusedSGD(backend.flat, lr=lr, momentum=momentum, weight_decay=weight_decay,
                       after_step=backend.after_optimizer_step, params=params)
        self._optimizers.append(opt)
        return opt

    def prepare_scheduler(self, scheduler, optimizer):
        s = GlobalRateScheduler(scheduler, optimizer, self.num_processes)
        self._schedulers.append(s)
        return s

    def register_for_checkpointing(self, *objs):
        for o in objs:
            if not hasattr(o, "state_dict") or not hasattr(o, "load_state_dict"):
                raise ValueError(f"{o} has no state_dict/load_state_dict")
            self._custom.append(o)

    # ------------------------------------------------------------------ collectives
    def gather(self, t: torch.Tensor) -> torch.Tensor:
        return self.state.all_gather_cat(t)

    def reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        return self.state.all_reduce_(t, op)

    def sync_buffers(self):
        """Rank-0 BN running statistics everywhere (before eval/save; DDP did it every forward, C3)."""
        for be in self._models:
            self.state.broadcast_tensors(list(be.model.buffers()))

    # ------------------------------------------------------------------ checkpoints
    def save_state(self, output_dir: str):
        self.sync_buffers()
        be = self._models[0]
        scaler = getattr(be, "scaler", None)
        _save_state(output_dir, be.model, self._optimizers, self._schedulers, self._custom, step=self.step,
                    rank=self.process_index, is_main=self.is_main_process, scaler=scaler,
                    barrier=self.wait_for_everyone, world_size=self.num_processes)
        self.wait_for_everyone()
        return output_dir

    def load_state(self, input_dir: str):
        be = self._models[0]
        ov = _load_state(input_dir, be.model, self._optimizers, self._schedulers, self._custom,
                         rank=self.process_index, scaler=getattr(be, "scaler", None))
        if hasattr(be, "reload_weights"):
            be.reload_weights()
        else:
            be.flat.rebind()
        self.step = ov.get("step", self.step)
        return ov

    # ------------------------------------------------------------------ tracking
    def init_trackers(self, project_name: str, config=None):
        self.trackers.init(project_name, config)

    def log(self, values, step: Optional[int] = None):
        self.trackers.log(values, step=step)

    def end_training(self):
        self.trackers.finish()
