"""Kinetics-style labeled video datasets (reference ``run.py:150-185``).

Directory layout ``root/<class_name>/<video>.{npy,mp4,avi,...}``; classes are the *sorted* sub-directory
names and a video's label is its class index (pytorchvideo ``LabeledVideoPaths.from_directory``).

Differences from the reference's ``LimitDataset(Kinetics(...))`` wrapper, all deliberate (README):

* map-style with an **exact** length: one item per (video, clip) of this rank's video shard, so the
  DataLoader, LR-schedule length and progress bar agree without the ``StopIteration`` truncation of R2;
  train = one random clip per video per epoch (``RandomClipSampler``), val = *every* uniform clip
  (``full_val=True``; the reference evaluates only ``num_videos`` of the ~4x more clips).
* the video sampler is resolved up front: ``DistributedSampler`` semantics (seed-0 shuffle, padding to a
  multiple of the world size, ``indices[rank::world]``) with ``set_epoch`` honoured (the reference never
  calls it), or a ``RandomSampler``-style permutation in a single process.
* in ``gpu`` mode items are *raw* uint8 frames (only the ``num_frames`` that UniformTemporalSubsample
  keeps) plus the sampled resize/crop/flip parameters; pixels are produced on device by the fused
  preprocessing kernel.  In ``cpu`` mode the item is the reference float transform output.
"""
from __future__ import annotations

import math
import os
import random
from dataclasses import dataclass
from fractions import Fraction
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

from .clip_sampling import ClipSampler, RandomClipSampler, UniformClipSampler
from .transforms import (ClipParams, pack_pathway_indices, reference_transform, sample_params,
                         uniform_temporal_indices)
from .video import FRAME_EXTENSIONS, VIDEO_EXTENSIONS, SyntheticVideo, Video, open_video


class LabeledVideoPaths:
    def __init__(self, paths_and_labels: List[Tuple[str, Dict]], classes: Optional[List[str]] = None):
        self._paths_and_labels = paths_and_labels
        self.classes = classes or []

    @classmethod
    def from_directory(cls, root: str) -> "LabeledVideoPaths":
        if not os.path.isdir(root):
            raise FileNotFoundError(f"{root} is not a directory")
        classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        items = []
        exts = VIDEO_EXTENSIONS + FRAME_EXTENSIONS
        for label, c in enumerate(classes):
            d = os.path.join(root, c)
            for f in sorted(os.listdir(d)):
                if os.path.splitext(f)[1].lower() in exts:
                    items.append((os.path.join(d, f), {"label": label}))
        return cls(items, classes)

    def __getitem__(self, i):
        return self._paths_and_labels[i]

    def __len__(self):
        return len(self._paths_and_labels)

    @property
    def num_videos(self) -> int:
        return len(self._paths_and_labels)

    @property
    def num_labels(self) -> int:
        """Distinct labels among the videos (reference run.py:185)."""
        return len({info["label"] for _, info in self._paths_and_labels})


class SyntheticVideoPaths(LabeledVideoPaths):
    """Virtual Kinetics-like corpus for runs without data (``--synthetic``)."""

    def __init__(self, num_videos: int, num_classes: int, num_frames: int = 300, height: int = 256,
                 width: int = 340, fps: float = 30.0, seed: int = 0, min_frames: Optional[int] = None):
        """``min_frames``: video lengths vary deterministically in [min_frames, num_frames] (as real Kinetics
        videos do, so the number of uniform validation clips differs per video and per rank); default: all
        ``num_frames`` long."""
        items = [(f"synthetic://{i}", {"label": i % num_classes}) for i in range(num_videos)]
        super().__init__(items, [f"class_{c}" for c in range(num_classes)])
        self.spec = (num_frames, height, width, fps)
        self.seed = seed
        self.min_frames = num_frames if min_frames is None else max(1, min(int(min_frames), num_frames))

    def frames_of(self, i: int) -> int:
        T = self.spec[0]
        span = T - self.min_frames + 1
        return T if span <= 1 else self.min_frames + (i * 7919 + self.seed * 104729) % span

    def open(self, i: int) -> Video:
        _, H, W, fps = self.spec
        return SyntheticVideo(f"video_{i}", self.seed * 7919 + i, self.frames_of(i), H, W, fps)


def distributed_video_indices(n: int, rank: int, world: int, seed: int = 0, epoch: int = 0,
                              shuffle: bool = True) -> List[int]:
    """torch ``DistributedSampler`` index math (shuffle with seed+epoch, pad to a multiple of world)."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    total = int(math.ceil(n / world)) * world
    pad = total - n
    if pad > 0:
        idx += (idx * math.ceil(pad / max(len(idx), 1)))[:pad]
    return idx[rank:total:world]


@dataclass
class ClipItem:
    video_index: int
    clip_index: int
    clip_start: Optional[Fraction] = None
    clip_end: Optional[Fraction] = None
    order: int = 0      # position in the epoch plan (keys the item's random draws)


class VideoClipDataset(Dataset):
    """Map-style clip dataset over one rank's shard of a labeled video corpus."""

    def __init__(self, videos: LabeledVideoPaths, clip_duration: float, training: bool, num_frames: int,
                 crop_size: int, slowfast_alpha: Optional[int], rank: int = 0, world: int = 1,
                 distributed: bool = False, seed: int = 0, full_val: bool = True, mode: str = "cpu",
                 min_scale: int = 256, max_scale: int = 320, mean=(0.45, 0.45, 0.45), std=(0.225, 0.225, 0.225)):
        self.videos = videos
        self.clip_duration = Fraction(clip_duration).limit_denominator(10000)
        self.training = training
        self.num_frames = num_frames
        self.crop = crop_size
        self.alpha = slowfast_alpha
        self.rank, self.world, self.distributed, self.seed = rank, world, distributed, seed
        self.full_val = full_val
        self.mode = mode
        self.min_scale, self.max_scale = min_scale, max_scale
        self.mean, self.std = mean, std
        self._durations: Dict[int, Fraction] = {}
        self.set_epoch(0)

    # ------------------------------------------------------------------ epoch plan
    def _open(self, i: int) -> Video:
        if isinstance(self.videos, SyntheticVideoPaths):
            return self.videos.open(i)
        return open_video(self.videos[i][0])

    def duration(self, i: int) -> Fraction:
        d = self._durations.get(i)
        if d is None:
            v = self._open(i)
            d = self._durations[i] = v.duration
            v.close()
        return d

    def set_epoch(self, epoch: int, force: bool = False):
        """Plan of ``epoch`` (deterministic in seed and epoch).  Re-planning the current epoch keeps the same
        ``items`` object (a reader that started on it ahead of time stays valid) unless ``force``."""
        if not force and getattr(self, "epoch", None) == epoch and getattr(self, "items", None) is not None:
            return
        self.epoch = epoch
        n = self.videos.num_videos
        if self.distributed:
            order = distributed_video_indices(n, self.rank, self.world, seed=self.seed, epoch=epoch,
                                              shuffle=self.training)
        elif self.training:
            g = torch.Generator()
            g.manual_seed(self.seed + epoch)
            order = torch.randperm(n, generator=g).tolist()
        else:
            order = list(range(n))
        items: List[ClipItem] = []
        if self.training:
            items = [ClipItem(v, 0, order=k) for k, v in enumerate(order)]
        else:
            for v in order:
                k = UniformClipSampler(self.clip_duration).num_clips(self.duration(v)) if self.full_val else 1
                d = self.clip_duration
                items += [ClipItem(v, c, c * d, (c + 1) * d) for c in range(k)]
        self.items = items

    def __len__(self):
        return len(self.items)

    # ------------------------------------------------------------------ items
    def item_rng(self, it: ClipItem):
        """(random.Random, torch.Generator) of one training item, seeded by (seed, epoch, rank, plan position, video):
        the clip start and the scale/crop/flip draws do not depend on global RNG state, so a reader that runs ahead
        of the training loop (next epoch prefetched before the epoch checkpoint, trainer.py) cannot shift them, and a
        run resumed from a checkpoint draws exactly what the uninterrupted run drew.  Same distributions as the
        reference's global-RNG draws (pytorchvideo RandomClipSampler, RandomShortSideScale / RandomCrop / flip)."""
        key = hash((int(self.seed), int(self.epoch), int(self.rank), int(it.order), int(it.video_index))) & (2 ** 62 - 1)
        g = torch.Generator()
        g.manual_seed(key)
        return random.Random(key), g

    def _clip_times(self, it: ClipItem, video: Video, rng=None):
        if it.clip_start is not None:
            return it.clip_start, it.clip_end
        info = RandomClipSampler(self.clip_duration, rng)(None, video.duration)
        return info.clip_start_sec, info.clip_end_sec

    def __getitem__(self, i: int):
        it = self.items[i]
        path, info = self.videos[it.video_index]
        video = self._open(it.video_index)
        rng, gen = self.item_rng(it) if self.training else (None, None)
        start, end = self._clip_times(it, video, rng)
        frame_idx = video.frame_indices(start, end)
        if not frame_idx:
            frame_idx = [max(video.num_frames - 1, 0)]
        sel = uniform_temporal_indices(len(frame_idx), self.num_frames).tolist()
        src = [frame_idx[j] for j in sel]
        sample = {"label": info["label"], "video_index": it.video_index, "clip_index": it.clip_index,
                  "aug_index": 0, "video_name": video.name}
        if self.mode == "gpu":
            # only the frames UniformTemporalSubsample keeps are read; tidx is the identity on them
            frames = video.read_frames(src)
            p = sample_params(self.num_frames, video.height, video.width, self.num_frames, self.crop,
                              self.training, self.min_scale, self.max_scale, generator=gen)
            sample["frames"] = torch.from_numpy(frames)
            sample["params"] = (p.rh, p.rw, p.top, p.left, int(p.flip))
        else:
            frames = torch.from_numpy(video.read_frames(src))
            p = sample_params(self.num_frames, video.height, video.width, self.num_frames, self.crop,
                              self.training, self.min_scale, self.max_scale, generator=gen)
            clip = reference_transform(frames, p, self.crop, self.mean, self.std)  # [3, T, S, S]
            if self.alpha:
                slow = clip.index_select(1, pack_pathway_indices(self.num_frames, self.alpha))
                sample["video"] = [slow, clip]
            else:
                sample["video"] = clip
        video.close()
        return sample


def collate_gpu(batch: Sequence[Dict]):
    """Collate raw clips: packed uint8 buffer + per-clip descriptors (clips may differ in H, W)."""
    T = batch[0]["frames"].shape[0]
    sizes = [int(b["frames"].numel()) for b in batch]
    packed = torch.empty(sum(sizes), dtype=torch.uint8)
    desc = torch.empty(len(batch), 10, dtype=torch.int32)
    off = 0
    for i, (b, n) in enumerate(zip(batch, sizes)):
        packed[off:off + n].copy_(b["frames"].reshape(-1))
        _, H, W, _ = b["frames"].shape
        rh, rw, top, left, flip = b["params"]
        desc[i] = torch.tensor([off & 0x7FFFFFFF, off >> 31, T, H, W, rh, rw, top, left, flip], dtype=torch.int32)
        off += n
    return {"frames": packed, "desc": desc, "num_frames": T,
            "label": torch.tensor([b["label"] for b in batch], dtype=torch.long),
            "video_index": torch.tensor([b["video_index"] for b in batch]),
            "clip_index": torch.tensor([b["clip_index"] for b in batch])}
