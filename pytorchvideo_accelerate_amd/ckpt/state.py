"""accelerate-compatible checkpoint directories (reference ``save_state``/``load_state``, SURVEY.md D11,
§3.5).

Layout of ``<dir>`` (same file names and formats as accelerate 1.x, so ``accelerate.Accelerator
.load_state`` can read ours and vice versa — pinned by ``tests/test_checkpoint.py``)::

    model.safetensors            model state_dict (pytorchvideo keys; no ``module.`` prefix, like a
                                 single-process accelerate save; a ``module.`` prefix is stripped on load)
    optimizer.bin                torch.save(SGD state_dict)  (momentum_buffer per param + param_groups)
    scheduler.bin                torch.save(scheduler state_dict)
    custom_checkpoint_{i}.pkl    registered objects' state_dict (the reference registers its scheduler)
    random_states_{rank}.pkl     {"step", "random_state", "numpy_random_seed", "torch_manual_seed",
                                  "torch_cuda_manual_seed"} — written by every rank
    scaler.pt                    GradScaler state (fp16 only)

Only the main process writes shared files; everything it reads back goes through ``weights_only=True``
loaders (safetensors / allow-listed torch.load).
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Sequence

import torch

from ..utils.misc import rng_state, safe_torch_load, set_rng_state

MODEL_FILE = "model.safetensors"
MODEL_BIN = "pytorch_model.bin"
OPTIMIZER_FILE = "optimizer.bin"
SCHEDULER_FILE = "scheduler.bin"
SCALER_FILE = "scaler.pt"


def _clean_for_safetensors(sd: Dict[str, torch.Tensor]) -> "OrderedDict[str, torch.Tensor]":
    out = OrderedDict()
    for k, v in sd.items():
        out[k] = v.detach().to("cpu").contiguous().clone()
    return out


def save_state(output_dir: str, model: torch.nn.Module, optimizers: Sequence = (), schedulers: Sequence = (),
               custom: Sequence = (), step: int = 0, rank: int = 0, is_main: bool = True, scaler=None) -> str:
    os.makedirs(output_dir, exist_ok=True)
    if is_main:
        from safetensors.torch import save_file
        save_file(_clean_for_safetensors(model.state_dict()), os.path.join(output_dir, MODEL_FILE),
                  metadata={"format": "pt"})
        for i, opt in enumerate(optimizers):
            name = OPTIMIZER_FILE if i == 0 else f"optimizer_{i}.bin"
            torch.save(opt.state_dict(), os.path.join(output_dir, name))
        for i, sch in enumerate(schedulers):
            name = SCHEDULER_FILE if i == 0 else f"scheduler_{i}.bin"
            torch.save(sch.state_dict(), os.path.join(output_dir, name))
        for i, obj in enumerate(custom):
            torch.save(obj.state_dict(), os.path.join(output_dir, f"custom_checkpoint_{i}.pkl"))
        if scaler is not None:
            torch.save(scaler.state_dict(), os.path.join(output_dir, SCALER_FILE))
    torch.save(rng_state(step), os.path.join(output_dir, f"random_states_{rank}.pkl"))
    return output_dir


def load_model_state(model: torch.nn.Module, input_dir: str, strict: bool = True):
    p = os.path.join(input_dir, MODEL_FILE)
    if os.path.exists(p):
        from safetensors.torch import load_file
        sd = load_file(p)
    else:
        sd = torch.load(os.path.join(input_dir, MODEL_BIN), map_location="cpu", weights_only=True)
    if any(k.startswith("module.") for k in sd):
        sd = OrderedDict((k[len("module."):] if k.startswith("module.") else k, v) for k, v in sd.items())
    missing, unexpected = model.load_state_dict(sd, strict=strict)
    return missing, unexpected


def load_state(input_dir: str, model: torch.nn.Module, optimizers: Sequence = (), schedulers: Sequence = (),
               custom: Sequence = (), rank: int = 0, map_location="cpu", scaler=None) -> Dict[str, Any]:
    """Load a checkpoint directory; returns overrides (``{"step": n}``) like accelerate."""
    load_model_state(model, input_dir)
    for i, opt in enumerate(optimizers):
        name = OPTIMIZER_FILE if i == 0 else f"optimizer_{i}.bin"
        opt.load_state_dict(torch.load(os.path.join(input_dir, name), map_location=map_location, weights_only=True))
    for i, sch in enumerate(schedulers):
        name = SCHEDULER_FILE if i == 0 else f"scheduler_{i}.bin"
        sch.load_state_dict(torch.load(os.path.join(input_dir, name), map_location="cpu", weights_only=True))
    n_custom = len([f for f in os.listdir(input_dir) if f.startswith("custom_checkpoint_")])
    if n_custom != len(custom):
        raise ValueError(f"found {n_custom} custom checkpoints but {len(custom)} objects were registered")
    for i, obj in enumerate(custom):
        obj.load_state_dict(torch.load(os.path.join(input_dir, f"custom_checkpoint_{i}.pkl"), map_location="cpu",
                                       weights_only=True))
    if scaler is not None and os.path.exists(os.path.join(input_dir, SCALER_FILE)):
        scaler.load_state_dict(torch.load(os.path.join(input_dir, SCALER_FILE), weights_only=True))
    out: Dict[str, Any] = {}
    rp = os.path.join(input_dir, f"random_states_{rank}.pkl")
    if os.path.exists(rp):
        try:
            st = safe_torch_load(rp)
            set_rng_state(st)
            out["step"] = st.get("step", 0)
        except Exception:  # pragma: no cover - mismatched numpy pickles
            pass
    return out


def latest_checkpoint(root: str) -> Optional[str]:
    """Most recently written ``epoch_*`` / ``step_*`` directory under ``root`` (the reference's dead
    "latest checkpoint" branch, ``run.py:208-212``, made real)."""
    if not os.path.isdir(root):
        return None
    cands = []
    for d in os.listdir(root):
        full = os.path.join(root, d)
        num = d[6:] if d.startswith("epoch_") else d[5:] if d.startswith("step_") else None
        if num is None or not num.isdigit() or not os.path.isdir(full):
            continue
        if not os.path.exists(os.path.join(full, MODEL_FILE)) and not os.path.exists(os.path.join(full, MODEL_BIN)):
            continue
        cands.append((os.path.getmtime(full), int(num), full))
    return max(cands)[2] if cands else None
