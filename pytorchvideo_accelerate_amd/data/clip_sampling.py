"""Clip samplers with pytorchvideo semantics (reference ``run.py:154,163`` → SURVEY.md D16).

* ``RandomClipSampler(d, rng=None)``: one clip per video per epoch, ``start ~ U(0, max(dur - d, 0))`` drawn with
  Python ``random`` (as pytorchvideo) — or with the given ``random.Random`` (the datasets pass a per-item generator,
  ``kinetics.VideoClipDataset.item_rng``), ``is_last_clip = True``.
* ``UniformClipSampler(d, stride=d)``: consecutive clips ``[k*stride, k*stride + d)``; a clip is the last
  one when the *next* clip would end past the video (``next_end - dur > eps``), so a 10 s video at
  d = 2.133 s yields 4 clips.
Times are ``fractions.Fraction`` like pytorchvideo so boundary decisions are exact.
"""
from __future__ import annotations

import random
from fractions import Fraction
from typing import NamedTuple, Optional


class ClipInfo(NamedTuple):
    clip_start_sec: Fraction
    clip_end_sec: Fraction
    clip_index: int
    aug_index: int
    is_last_clip: bool


class ClipSampler:
    def __init__(self, clip_duration):
        self._clip_duration = Fraction(clip_duration)
        self._current_clip_index = 0
        self._current_aug_index = 0

    def reset(self):
        self._current_clip_index = 0
        self._current_aug_index = 0

    def __call__(self, last_clip_end_time, video_duration, annotation=None) -> ClipInfo:
        raise NotImplementedError


class RandomClipSampler(ClipSampler):
    def __init__(self, clip_duration, rng: Optional[random.Random] = None):
        super().__init__(clip_duration)
        self._rng = rng

    def __call__(self, last_clip_end_time, video_duration, annotation=None) -> ClipInfo:
        max_start = max(Fraction(video_duration) - self._clip_duration, 0)
        start = Fraction((self._rng or random).uniform(0, float(max_start)))
        return ClipInfo(start, start + self._clip_duration, 0, 0, True)


class UniformClipSampler(ClipSampler):
    def __init__(self, clip_duration, stride=None, backpad_last: bool = False, eps: float = 1e-6):
        super().__init__(clip_duration)
        self._stride = Fraction(stride) if stride is not None else self._clip_duration
        self._backpad_last = backpad_last
        self._eps = eps

    def _start_end(self, last_end, video_duration):
        delta = self._stride - self._clip_duration
        last_end = -delta if last_end is None else Fraction(last_end)
        start = Fraction(last_end + delta)
        end = Fraction(start + self._clip_duration)
        if self._backpad_last:
            buffer_amount = max(0, end - Fraction(video_duration))
            start -= buffer_amount
            start = max(0, start)
            end = Fraction(start + self._clip_duration)
        return start, end

    def __call__(self, last_clip_end_time, video_duration, annotation=None) -> ClipInfo:
        start, end = self._start_end(last_clip_end_time, video_duration)
        _, next_end = self._start_end(end, video_duration)
        if self._backpad_last:
            is_last = abs(next_end - end) < self._eps
        else:
            is_last = (next_end - Fraction(video_duration)) > self._eps
        idx = self._current_clip_index
        self._current_clip_index += 1
        if is_last:
            self.reset()
        return ClipInfo(start, end, idx, 0, is_last)

    def num_clips(self, video_duration) -> int:
        """Number of clips this sampler yields for one video (exact-count val iteration)."""
        n, last = 0, None
        while True:
            info = self(last, video_duration)
            n += 1
            last = info.clip_end_sec
            if info.is_last_clip:
                return n


def make_clip_sampler(sampling_type: str, *args) -> ClipSampler:
    if sampling_type == "random":
        return RandomClipSampler(*args)
    if sampling_type == "uniform":
        return UniformClipSampler(*args)
    raise NotImplementedError(f"{sampling_type} clip sampling not supported")
