"""The alternate arms of finished A/B experiments, behind ONE knob: ``PVA_ARMS``.

Every default below is the arm that won its measurement (the profile directory says where); the shipped
configuration is the default of every arm.  ``PVA_ARMS="stem_pair=0,side_fuse=0"`` selects other arms — for the
tests that keep the alternate kernels numerically honest and for A/B reruns.  An unknown arm name raises, so a typo
cannot silently run the default.  The native stem kernels read the same variable (``csrc/kernels/stem_s2d.hip``).

Operational knobs (not arms) stay separate environment variables and are listed in README "Configuration":
PVA_AUTOBUILD, PVA_TUNE_CACHE, PVA_TUNE_LOG, PVA_COMM, PVA_DIST_BACKEND, PVA_FORCE_GRADSYNC, PVA_RCCL_LIB,
PVA_AUTO_RESUME, PVA_FAULT, PVA_PRETRAINED, PVA_ROCTX.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Union

Value = Union[int, str, None]

# name -> (default, where the default was decided)
DEFAULTS: Dict[str, tuple] = {
    # autotuner candidate families (ops/tune.py)
    "autotune": (1, "r1: heuristic configs only when 0"),
    "conv_direct": (1, "r3_knobs"),
    "conv_dma": (1, "r3_knobs"),
    "conv_pw": (1, "r2_final"),
    "conv_halo": (1, "r3_halo"),
    "conv_halo_d": (1, "r6_halo: double-buffered 64-channel halo conv as a tuner candidate"),
    "conv_big_half": (1, "r4_big_half"),
    "conv_pf": (1, "r5_lab"),
    "conv_pw_w4": (1, "r5_lateral"),
    "pw_kinds": (None, "debugging aid: restrict the pointwise kernel to these launch kinds"),
    "tune_reps": (3, "r4_tune_reps"),
    "tune_top": (3, "r4_tune_reps"),
    # executor (models/fused.py)
    "streams": (1, "r2_final: two-stream execution"),
    "side_priority": (0, "r5_hwq"),
    "side_fuse": (1, "r5_side"),
    "lateral_bwd": (1, "r5_lateral"),
    "fold_slabs": (1, "r4_regress"),
    "bn_fold": (1, "r2_pmc_final"),
    "bn_fold_min_c": (16, "r4_fold"),
    "bn_fold1": (1, "r3_fold1"),
    "bn_fold_exact_below": (32, "r4_fold (scripts/diag_ms_fold.py @ a59cdac)"),
    "narrow_bwd": (1, "r5_narrow"),
    "narrow_splits": (1024, "r5_narrow"),
    "narrow_fold": (1, "r5_narrow"),
    # fp32 path (models/native32.py): bf16 pieces per fp32 conv operand — 3: fp32 accuracy (6 MFMA products),
    # 2: ~16-bit operands (3 products, 2x the throughput; tests/test_native32_gpu.py measures both)
    "f32_pieces": (3, "r6_f32"),
    # stem kernels (csrc/kernels/stem_s2d.hip reads these itself)
    "stem_pair": (1, "r4_stem"),
    "stem_perm": (1, "r5_end"),
    "stem_roll": (1, "r5_stem_roll"),
    "stem_async": (1, "r5_stem_roll"),
}


def _parse(spec: str) -> Dict[str, str]:
    out = {}
    for item in spec.split(","):
        item = item.strip()
        if not item:
            continue
        if "=" not in item:
            raise ValueError(f"PVA_ARMS entry {item!r} is not name=value")
        k, v = item.split("=", 1)
        k = k.strip()
        if k not in DEFAULTS:
            raise ValueError(f"PVA_ARMS: unknown arm {k!r} (known: {', '.join(sorted(DEFAULTS))})")
        out[k] = v.strip()
    return out


def arm(name: str) -> Value:
    """The selected value of arm ``name`` (its default unless PVA_ARMS overrides it)."""
    dflt = DEFAULTS[name][0]
    v = _parse(os.environ.get("PVA_ARMS", "")).get(name)
    if v is None:
        return dflt
    if isinstance(dflt, int):
        return int(v)
    return v


def on(name: str) -> bool:
    return bool(arm(name))


def arms_spec(**kw) -> str:
    """``PVA_ARMS`` value selecting the given arms on top of the current ones (tests: monkeypatch.setenv)."""
    cur = _parse(os.environ.get("PVA_ARMS", ""))
    for k, v in kw.items():
        if k not in DEFAULTS:
            raise ValueError(f"unknown arm {k!r}")
        cur[k] = str(int(v) if isinstance(v, bool) else v)
    return ",".join(f"{k}={v}" for k, v in cur.items())


def selected() -> Dict[str, Optional[Value]]:
    """Every arm with a non-default value (recorded in tune-table identities and logs)."""
    return {k: arm(k) for k in DEFAULTS if arm(k) != DEFAULTS[k][0]}
