"""Video transforms: exact index/rounding math of the reference pipeline + the on-device executor.

Reference pipeline (``run.py:68-102``)::

    UniformTemporalSubsample(num_frames) → Div255 → Normalize(0.45, 0.225)
      train: RandomShortSideScale(256, 320) → RandomCrop(crop) → RandomHorizontalFlip(0.5)
      val:   ShortSideScale(256) → CenterCrop(crop)
    → PackPathway(alpha)  (SlowFast only)

Host side we only *sample the parameters* (frame indices, resize size, crop box, flip) with the same
RNG streams the reference uses (torch RNG for scale/crop/flip); the pixels are produced by ONE fused
HIP kernel per pathway (``video_preprocess``) straight from the decoded uint8 frames: temporal gather →
bilinear resize (``align_corners=False``) → crop → flip → normalise → bf16 NDHWC (RGB + zero pad
channel).  Normalisation commutes with the resize exactly in real arithmetic (bilinear weights sum to
1), so resizing raw uint8 then normalising is the reference result up to float rounding.

A pure-torch implementation of the same chain (``reference_transform``) is kept for CPU runs and as the
test oracle.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

MEAN = (0.45, 0.45, 0.45)
STD = (0.225, 0.225, 0.225)


def uniform_temporal_indices(t_src: int, num: int) -> torch.Tensor:
    """pytorchvideo UniformTemporalSubsample: linspace(0, T-1, n).clamp(0, T-1).long()."""
    return torch.linspace(0, t_src - 1, num).clamp(0, t_src - 1).long()


def pack_pathway_indices(t: int, alpha: int) -> torch.Tensor:
    """Reference PackPathway (run.py:59-63): linspace(0, T-1, T // alpha).long() (truncation)."""
    return torch.linspace(0, t - 1, t // alpha).long()


def short_side_scale_size(h: int, w: int, size: int) -> Tuple[int, int]:
    """pytorchvideo short_side_scale output size: short side = size, long side = floor(long/short*size)."""
    if w < h:
        return int(math.floor((float(h) / w) * size)), size
    return size, int(math.floor((float(w) / h) * size))


def center_crop_box(h: int, w: int, s: int) -> Tuple[int, int]:
    """torchvision CenterCrop offsets: round((H - s) / 2)."""
    return int(round((h - s) / 2.0)), int(round((w - s) / 2.0))


@dataclass
class ClipParams:
    tidx: List[int]      # source frame index per output (fast) frame
    rh: int
    rw: int
    top: int
    left: int
    flip: bool


def sample_params(t_src: int, h: int, w: int, num_frames: int, crop: int, training: bool,
                  min_scale: int = 256, max_scale: int = 320, flip_p: float = 0.5,
                  generator: Optional[torch.Generator] = None) -> ClipParams:
    tidx = uniform_temporal_indices(t_src, num_frames).tolist()
    if training:
        size = int(torch.randint(min_scale, max_scale + 1, (1,), generator=generator).item())
    else:
        size = min_scale
    rh, rw = short_side_scale_size(h, w, size)
    if training:
        top = int(torch.randint(0, rh - crop + 1, size=(1,), generator=generator).item())
        left = int(torch.randint(0, rw - crop + 1, size=(1,), generator=generator).item())
        flip = bool(torch.rand(1, generator=generator).item() < flip_p)
    else:
        top, left = center_crop_box(rh, rw, crop)
        flip = False
    return ClipParams(tidx, rh, rw, top, left, flip)


def reference_transform(frames_u8: torch.Tensor, p: ClipParams, crop: int, mean=MEAN, std=STD) -> torch.Tensor:
    """Pure-torch oracle. frames_u8: [T_src, H, W, 3] uint8 -> float [3, T, crop, crop] (reference order)."""
    x = frames_u8.permute(3, 0, 1, 2).float()                       # C,T,H,W
    x = x.index_select(1, torch.tensor(p.tidx, dtype=torch.long))    # UniformTemporalSubsample
    x = x / 255.0                                                    # Div255
    m = torch.tensor(mean).view(3, 1, 1, 1)
    s = torch.tensor(std).view(3, 1, 1, 1)
    x = (x - m) / s                                                  # Normalize
    x = F.interpolate(x, size=(p.rh, p.rw), mode="bilinear", align_corners=False)  # (N=C, C=T) trick
    x = x[..., p.top:p.top + crop, p.left:p.left + crop]
    if p.flip:
        x = x.flip(-1)
    return x


class GpuClipBatch:
    """Runs the fused preprocess kernel for a batch of decoded clips (same source shape)."""

    def __init__(self, device, num_frames: int, crop: int, alpha: Optional[int], mean=MEAN, std=STD,
                 s2d: bool = False, dtype: torch.dtype = torch.bfloat16):
        """``dtype``: the executor's 16-bit compute type (bf16, or fp16 for ``--mixed_precision fp16``)."""
        from ..ops._ext import require
        self.C = require()
        self.dtype = dtype
        self.s2d = s2d  # space-to-depth output for the direct stem kernels (C = 16 at S/2 x S/2)
        self.device = torch.device(device)
        self.T, self.S, self.alpha = num_frames, crop, alpha
        self.mean, self.std = list(mean), list(std)
        self.slow_sel = pack_pathway_indices(num_frames, alpha) if alpha else None
        self._out = {}

    def _buf(self, key, shape):
        t = self._out.get(key)
        if t is None or tuple(t.shape) != tuple(shape):
            t = torch.empty(shape, device=self.device, dtype=self.dtype)
            self._out[key] = t
        return t

    def _act(self, buf, B, T):
        from ..ops.conv import Act
        if self.s2d:
            return Act(buf.view(-1, 16), B, T, self.S // 2, self.S // 2)
        return Act(buf, B, T, self.S, self.S)

    def _slow_of(self, device):
        """[T] int32: the slow frame each frame also feeds (-1: none); None if the selection repeats a frame."""
        key = ("slow_of", device)
        if key not in self._out:
            sel = self.slow_sel.tolist()
            m = None
            if len(set(sel)) == len(sel):
                m = torch.full((self.T,), -1, dtype=torch.int32)
                for s, t in enumerate(sel):
                    m[t] = s
                m = m.to(device)
            self._out[key] = m
        return self._out[key]

    def _run(self, frames: torch.Tensor, desc: torch.Tensor, tidx: torch.Tensor):
        B = desc.shape[0]
        fast = self._buf("fast", (B * self.T * self.S * self.S, 4))
        if not self.alpha:
            self.C.video_preprocess(frames, desc, tidx, self.T, self.S, self.mean, self.std, fast, self.s2d)
            return [self._act(fast, B, self.T)]
        Ts = len(self.slow_sel)
        slow = self._buf("slow", (B * Ts * self.S * self.S, 4))
        slow_of = self._slow_of(tidx.device)
        if slow_of is not None:
            # one pass: the slow frames are a subset of the fast ones, written from the same cells
            self.C.video_preprocess(frames, desc, tidx, self.T, self.S, self.mean, self.std, fast, self.s2d,
                                    slow_of, slow, Ts)
        else:
            sel = self._out.get(("sel", tidx.device))
            if sel is None:
                sel = self._out[("sel", tidx.device)] = self.slow_sel.to(tidx.device)
            stidx = tidx.index_select(1, sel).contiguous()
            self.C.video_preprocess(frames, desc, stidx, Ts, self.S, self.mean, self.std, slow, self.s2d)
            self.C.video_preprocess(frames, desc, tidx, self.T, self.S, self.mean, self.std, fast, self.s2d)
        return [self._act(slow, B, Ts), self._act(fast, B, self.T)]

    def __call__(self, frames: torch.Tensor, params: Sequence[ClipParams]):
        """frames: [B, T_src, H, W, 3] uint8 on device (same source shape) -> [slow, fast] or [clip] Acts."""
        B, Ts, H, W, _ = frames.shape
        per = Ts * H * W * 3
        desc = torch.tensor([[(b * per) & 0x7FFFFFFF, (b * per) >> 31, Ts, H, W, p.rh, p.rw, p.top, p.left,
                              int(p.flip)] for b, p in enumerate(params)], dtype=torch.int32)
        tidx = torch.tensor([p.tidx for p in params], dtype=torch.int32)
        pin = self.device.type == "cuda"
        if pin:
            desc, tidx = desc.pin_memory(), tidx.pin_memory()
        return self._run(frames, desc.to(self.device, non_blocking=pin), tidx.to(self.device, non_blocking=pin))

    def from_packed(self, frames: torch.Tensor, desc: torch.Tensor, num_frames: int):
        """Loader path: packed, already temporally-subsampled clips (tidx = identity)."""
        B = desc.shape[0]
        key = ("tidx", B, num_frames)
        tidx = self._out.get(key)
        if tidx is None:   # device-resident identity index (no pageable H2D copy per batch)
            tidx = self._out[key] = torch.arange(num_frames, dtype=torch.int32).repeat(B, 1).to(self.device)
        return self._run(frames, desc.to(self.device, non_blocking=True), tidx)
