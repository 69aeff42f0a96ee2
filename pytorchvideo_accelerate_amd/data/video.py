"""Pluggable video decoders.

The image has no FFmpeg/PyAV/decord, so decoding is an interface with three back-ends:

* :class:`RawFramesVideo` — pre-decoded uint8 frames ``<name>.npy`` ``[T, H, W, 3]`` (memory-mapped,
  ``allow_pickle=False``) with an optional ``<name>.json`` ``{"fps": 30}`` sidecar.  Clip reads touch only
  the frames needed; the native reader (``csrc/runtime/clip_reader.cpp``) copies them straight into
  pinned host memory with a thread pool.
* :class:`SyntheticVideo` — deterministic pseudo-random frames (benchmark / tests; never all-zero).
* :class:`PyAVVideo` — H.264/MPEG-4 via PyAV when ``av`` is importable (not in this image; gated).

``get_clip(start, end)`` returns the frames whose timestamps ``i / fps`` lie in ``[start, end)`` as
``uint8 [T, H, W, 3]`` (pytorchvideo ``EncodedVideo.get_clip`` semantics; T varies with the source fps).
"""
from __future__ import annotations

import json
import math
import os
from fractions import Fraction
from typing import Optional, Sequence

import numpy as np

VIDEO_EXTENSIONS = (".mp4", ".avi", ".mkv", ".webm", ".mov")
FRAME_EXTENSIONS = (".npy",)


def frame_range(start, end, fps: float, num_frames: int):
    """Indices i with start <= i/fps < end, clipped to the video."""
    a = max(int(math.ceil(float(Fraction(start)) * fps - 1e-9)), 0)
    b = min(int(math.ceil(float(Fraction(end)) * fps - 1e-9)), num_frames)
    return a, max(a, b)


class Video:
    name: str
    fps: float
    num_frames: int
    height: int
    width: int

    @property
    def duration(self) -> Fraction:
        return Fraction(self.num_frames) / Fraction(self.fps).limit_denominator(1000)

    def frame_indices(self, start, end):
        a, b = frame_range(start, end, self.fps, self.num_frames)
        return list(range(a, b))

    def read_frames(self, idx: Sequence[int]) -> np.ndarray:
        raise NotImplementedError

    def get_clip(self, start, end) -> Optional[np.ndarray]:
        idx = self.frame_indices(start, end)
        if not idx:
            return None
        return self.read_frames(idx)

    def close(self):
        pass


class RawFramesVideo(Video):
    def __init__(self, path: str, fps: Optional[float] = None):
        self.path = path
        self.name = os.path.splitext(os.path.basename(path))[0]
        self._arr = np.load(path, mmap_mode="r", allow_pickle=False)
        if self._arr.ndim != 4 or self._arr.shape[-1] != 3 or self._arr.dtype != np.uint8:
            raise ValueError(f"{path}: expected uint8 [T,H,W,3], got {self._arr.dtype} {self._arr.shape}")
        side = os.path.splitext(path)[0] + ".json"
        if fps is None and os.path.exists(side):
            with open(side) as fh:
                fps = float(json.load(fh).get("fps", 30))
        self.fps = float(fps or 30)
        self.num_frames, self.height, self.width = (int(v) for v in self._arr.shape[:3])

    @property
    def data_offset(self) -> int:
        return int(self._arr.offset) if hasattr(self._arr, "offset") else 0

    def read_frames(self, idx):
        return np.ascontiguousarray(self._arr[np.asarray(idx)])

    def close(self):
        self._arr = None


class SyntheticVideo(Video):
    """Deterministic uint8 noise video (per-video seed)."""

    def __init__(self, name: str, seed: int, num_frames: int = 300, height: int = 256, width: int = 340,
                 fps: float = 30.0):
        self.name, self.seed = name, seed
        self.num_frames, self.height, self.width, self.fps = num_frames, height, width, fps

    def read_frames(self, idx):
        out = np.empty((len(idx), self.height, self.width, 3), dtype=np.uint8)
        for j, i in enumerate(idx):
            rng = np.random.default_rng((self.seed * 1000003 + int(i)) & 0xFFFFFFFF)
            out[j] = rng.integers(1, 256, size=(self.height, self.width, 3), dtype=np.uint8)
        return out


class PyAVVideo(Video):  # pragma: no cover - PyAV is not installed in this image
    def __init__(self, path: str):
        import av  # noqa: F401
        self.path = path
        self.name = os.path.splitext(os.path.basename(path))[0]
        self._c = av.open(path)
        st = self._c.streams.video[0]
        self.fps = float(st.average_rate or 30)
        self.num_frames = int(st.frames or round(float(st.duration * st.time_base) * self.fps))
        self.height, self.width = st.codec_context.height, st.codec_context.width

    def read_frames(self, idx):
        want = set(idx)
        frames = []
        self._c.seek(0)
        for i, fr in enumerate(self._c.decode(video=0)):
            if i in want:
                frames.append(fr.to_ndarray(format="rgb24"))
            if i >= max(idx):
                break
        return np.stack(frames)

    def close(self):
        self._c.close()


def pyav_available() -> bool:
    try:
        import av  # noqa: F401
        return True
    except Exception:
        return False


def open_video(path: str) -> Video:
    ext = os.path.splitext(path)[1].lower()
    if ext in FRAME_EXTENSIONS:
        return RawFramesVideo(path)
    if ext in VIDEO_EXTENSIONS:
        if not pyav_available():
            raise RuntimeError(f"cannot decode {path}: PyAV/FFmpeg is not installed; convert videos to "
                               "uint8 .npy frames (see README) or use --synthetic")
        return PyAVVideo(path)
    raise ValueError(f"unsupported video file {path}")
