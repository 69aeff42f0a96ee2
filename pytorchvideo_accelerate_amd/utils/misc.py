"""Seeding, RNG-state capture and small helpers (accelerate ``set_seed`` / RNG checkpoint parity,
SURVEY.md D13 / D11)."""
from __future__ import annotations

import random
from typing import Any, Dict

import numpy as np
import torch


def set_seed(seed: int) -> None:
    """Seed python ``random``, numpy, torch CPU and every GPU (``accelerate.utils.set_seed``)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def rng_state(step: int) -> Dict[str, Any]:
    """RNG snapshot with accelerate's ``random_states_{rank}.pkl`` keys."""
    st = {
        "step": step,
        "random_state": random.getstate(),
        "numpy_random_seed": np.random.get_state(),
        "torch_manual_seed": torch.get_rng_state(),
    }
    if torch.cuda.is_available():
        st["torch_cuda_manual_seed"] = torch.cuda.get_rng_state_all()
    return st


def set_rng_state(st: Dict[str, Any]) -> None:
    random.setstate(st["random_state"])
    np.random.set_state(st["numpy_random_seed"])
    torch.set_rng_state(st["torch_manual_seed"])
    if torch.cuda.is_available() and "torch_cuda_manual_seed" in st:
        cur = torch.cuda.get_rng_state_all()
        vals = st["torch_cuda_manual_seed"]
        torch.cuda.set_rng_state_all(list(vals)[: len(cur)])


def safe_torch_load(path, map_location="cpu"):
    """``torch.load(weights_only=True)`` with the numpy types of RNG snapshots allow-listed.

    Never unpickles arbitrary objects (accelerate's ``load`` does the same allow-listing)."""
    import torch.serialization as ser
    allow = [np.ndarray, np.dtype]
    core = getattr(np, "_core", None)
    if core is None:  # numpy < 2
        core = np.core  # type: ignore[attr-defined]
    allow.append(core.multiarray._reconstruct)
    for name in ("UInt32DType", "Int64DType", "Float64DType", "Float32DType", "BoolDType"):
        t = getattr(np.dtypes, name, None) if hasattr(np, "dtypes") else None
        if t is not None:
            allow.append(t)
    with ser.safe_globals(allow):
        return torch.load(path, map_location=map_location, weights_only=True)


def fault_at(kind: str):
    """Fault-injection test hook ``PVA_FAULT="<kind>=N"`` (kinds: ``step`` — fail once when global step N completes,
    engine/trainer.py; ``save`` — crash inside the save of step N, ckpt/state.py).  Returns N or None."""
    import os
    spec = os.environ.get("PVA_FAULT", "")
    for item in spec.split(","):
        k, _, v = item.partition("=")
        if k.strip() == kind and v.strip():
            return int(v)
    return None
