"""Debug aids (SURVEY.md §5 race detection / failure detection).

* :class:`GradChecker` — NaN/Inf detector on the flat fp32 gradient buffer: one fused ``isfinite`` reduction
  per check; on failure it names the offending parameters (flat-buffer spans -> module names).
* :func:`debug_env` — environment for localising GPU faults: serialised kernel launches
  (``AMD_SERIALIZE_KERNEL=3``, ``AMD_SERIALIZE_COPY=3``) and synchronous HIP errors (``HIP_LAUNCH_BLOCKING``).
* Determinism: ``FusedNet(deterministic=True)`` (bitwise-reproducible gradients: slab wgrad reduction,
  generic stems); BN statistics are always reduced in a fixed order without float atomics.
* Host sanitizers: ``tests/test_native_sanitizers.py`` builds the native clip reader with TSan and
  ASan+UBSan.  GPU-side sanitizers are not available on the MI355X pool.
"""
from __future__ import annotations

import os
from typing import Dict, List

import torch


class GradChecker:
    """Check a :class:`~pytorchvideo_accelerate_amd.models.fused.FlatParams` gradient buffer for NaN/Inf."""

    def __init__(self, flat):
        self.flat = flat

    def bad_params(self) -> List[str]:
        g = self.flat.grad
        if bool(torch.isfinite(g).all()):
            return []
        bad = []
        for name, p, off in zip(self.flat.names, self.flat.params, self.flat.offsets):
            if not bool(torch.isfinite(g[off:off + p.numel()]).all()):
                bad.append(name)
        return bad

    def check(self, step: int = -1) -> None:
        bad = self.bad_params()
        if bad:
            raise FloatingPointError(f"non-finite gradients at step {step} in {len(bad)} parameter(s): "
                                     + ", ".join(bad[:8]) + (" ..." if len(bad) > 8 else ""))


def debug_env(serialize: bool = True) -> Dict[str, str]:
    """Environment variables for a fault-localisation run (apply before the GPU is initialised)."""
    env = {"HIP_LAUNCH_BLOCKING": "1"}
    if serialize:
        env.update({"AMD_SERIALIZE_KERNEL": "3", "AMD_SERIALIZE_COPY": "3"})
    return env


def apply_debug_env(serialize: bool = True) -> None:
    for k, v in debug_env(serialize).items():
        os.environ.setdefault(k, v)
