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

    .pva_complete                completion marker (JSON), written last

Saves are atomic: the main process writes the shared files into ``<dir>.tmp``, fsyncs them and renames the
directory into place (``os.replace``); after a barrier every rank writes its RNG file (temp file + rename), and
after a second barrier the main process writes the completion marker.  ``latest_checkpoint`` (auto-resume after an
elastic restart) only considers directories with that marker, so a crash in the middle of a save resumes from the
previous complete checkpoint instead of failing on a half-written one (``PVA_FAULT=save=N`` injects such a crash
into the save of global step N: ``tests/test_checkpoint.py``).

Only the main process writes shared files; everything it reads back goes through ``weights_only=True``
loaders (safetensors / allow-listed torch.load).
"""
from __future__ import annotations

import json
import os
import shutil
from collections import OrderedDict
from typing import Any, Callable, Dict, List, Optional, Sequence

import torch

from ..utils.misc import rng_state, safe_torch_load, set_rng_state

MODEL_FILE = "model.safetensors"
MODEL_BIN = "pytorch_model.bin"
OPTIMIZER_FILE = "optimizer.bin"
SCHEDULER_FILE = "scheduler.bin"
SCALER_FILE = "scaler.pt"
COMPLETE_FILE = ".pva_complete"


class InjectedSaveFault(RuntimeError):
    """Raised by ``PVA_FAULT=save=N`` (crash in the middle of a checkpoint save; test hook)."""


def _fsync_path(path: str):
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def _atomic_torch_save(obj, path: str):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    _fsync_path(tmp)
    os.replace(tmp, path)


def _maybe_fault_in_save(step: int, output_dir: str):
    from ..utils.misc import fault_at
    at = fault_at("save")
    if at is None or step != at:
        return
    marker = os.path.join(os.path.dirname(output_dir) or ".", f".save_fault_injected_{os.environ.get('RANK', '0')}")
    if os.path.exists(marker):
        return
    open(marker, "w").close()
    raise InjectedSaveFault(f"injected fault while saving {output_dir}")


def _clean_for_safetensors(sd: Dict[str, torch.Tensor]) -> "OrderedDict[str, torch.Tensor]":
    out = OrderedDict()
    for k, v in sd.items():
        out[k] = v.detach().to("cpu").contiguous().clone()
    return out


def save_state(output_dir: str, model: torch.nn.Module, optimizers: Sequence = (), schedulers: Sequence = (),
               custom: Sequence = (), step: int = 0, rank: int = 0, is_main: bool = True, scaler=None,
               barrier: Optional[Callable[[], None]] = None, world_size: int = 1) -> str:
    """Atomic save (module docstring).  ``barrier``: the process-group barrier (every rank calls this)."""
    barrier = barrier or (lambda: None)
    output_dir = os.path.normpath(output_dir)
    if is_main:
        from safetensors.torch import save_file
        tmp = output_dir + ".tmp"
        shutil.rmtree(tmp, ignore_errors=True)
        os.makedirs(tmp)
        files = []

        def put(name, obj):
            torch.save(obj, os.path.join(tmp, name))
            files.append(name)
        save_file(_clean_for_safetensors(model.state_dict()), os.path.join(tmp, MODEL_FILE), metadata={"format": "pt"})
        files.append(MODEL_FILE)
        _maybe_fault_in_save(step, output_dir)
        for i, opt in enumerate(optimizers):
            put(OPTIMIZER_FILE if i == 0 else f"optimizer_{i}.bin", opt.state_dict())
        for i, sch in enumerate(schedulers):
            put(SCHEDULER_FILE if i == 0 else f"scheduler_{i}.bin", sch.state_dict())
        for i, obj in enumerate(custom):
            put(f"custom_checkpoint_{i}.pkl", obj.state_dict())
        if scaler is not None:
            put(SCALER_FILE, scaler.state_dict())
        for f in files:
            _fsync_path(os.path.join(tmp, f))
        _fsync_path(tmp)
        old = None
        if os.path.isdir(output_dir):   # re-save into an existing directory: swap, then drop the old one
            old = output_dir + ".old"
            shutil.rmtree(old, ignore_errors=True)
            os.replace(output_dir, old)
        os.replace(tmp, output_dir)
        _fsync_path(os.path.dirname(output_dir) or ".")
        if old is not None:
            shutil.rmtree(old, ignore_errors=True)
    barrier()
    if not is_main:   # a node that does not share the main process's filesystem (accelerate: every rank creates it)
        os.makedirs(output_dir, exist_ok=True)
    _atomic_torch_save(rng_state(step), os.path.join(output_dir, f"random_states_{rank}.pkl"))
    barrier()
    if is_main:
        mk = os.path.join(output_dir, COMPLETE_FILE)
        with open(mk + ".tmp", "w") as f:
            json.dump({"step": int(step), "world_size": int(world_size)}, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(mk + ".tmp", mk)
        _fsync_path(output_dir)
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


def is_complete(path: str) -> bool:
    """Whether ``path`` holds a checkpoint whose save finished (completion marker present)."""
    return os.path.isfile(os.path.join(path, COMPLETE_FILE))


def latest_checkpoint(root: str) -> Optional[str]:
    """Most recently written COMPLETE ``epoch_*`` / ``step_*`` directory under ``root`` (the reference's dead
    "latest checkpoint" branch, ``run.py:208-212``, made real).  Directories without the completion marker (a save
    that crashed, or a directory another tool wrote: pass those to ``--resume_from_checkpoint`` explicitly) are
    skipped."""
    if not os.path.isdir(root):
        return None
    cands = []
    for d in os.listdir(root):
        full = os.path.join(root, d)
        num = d[6:] if d.startswith("epoch_") else d[5:] if d.startswith("step_") else None
        if num is None or not num.isdigit() or not os.path.isdir(full):
            continue
        if not is_complete(full):
            continue
        cands.append((os.path.getmtime(full), int(num), full))
    return max(cands)[2] if cands else None
