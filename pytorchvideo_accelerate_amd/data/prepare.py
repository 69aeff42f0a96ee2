"""Kinetics data preparation for this framework's raw-frame format (reference ``README.md:35-56``).

The reference downloads Kinetics-700 with torchvision (``root/{train,val}/<class>/<video>.mp4``) and decodes
mp4 on the fly with PyAV.  This image has no decoder, so the supported training format is **pre-decoded
raw frames** in the same directory layout:

    <root>/{train,val}/<class_name>/<video>.npy     uint8 [T, H, W, 3] (RGB, C-contiguous, np.save, no pickle)
    <root>/{train,val}/<class_name>/<video>.json    {"fps": <source frame rate>}   (optional, default 30)

Labels are the index of ``class_name`` in the sorted class folders (``LabeledVideoPaths.from_directory``);
clip sampling uses the real timestamps ``i / fps`` exactly like decoding the mp4 would.  Short side ~256-320
(Kinetics' usual 340x256 re-encodes) keeps files small and matches the train transform's 256-320 scale range.

    python -m pytorchvideo_accelerate_amd.data.prepare convert --src /data/kinetics --dst /data/k700_frames \
        [--short_side 320] [--workers 8]        # needs PyAV (``pip install av``) on the conversion host
    python -m pytorchvideo_accelerate_amd.data.prepare synthetic --dst /tmp/fake_k --classes 4 --videos 3
    python -m pytorchvideo_accelerate_amd.data.prepare check --root /data/k700_frames
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import sys
from typing import Dict, List, Tuple

import numpy as np

from .video import FRAME_EXTENSIONS, VIDEO_EXTENSIONS, RawFramesVideo, pyav_available

SPLITS = ("train", "val")


def _resize_short_side(frames: np.ndarray, short: int) -> np.ndarray:
    """Bilinear (align_corners=False) short-side resize of uint8 [T,H,W,3] on the CPU via torch."""
    import torch
    import torch.nn.functional as F
    T, H, W, _ = frames.shape
    if min(H, W) == short:
        return frames
    if H < W:
        nh, nw = short, int(W * short / H)
    else:
        nh, nw = int(H * short / W), short
    x = torch.from_numpy(frames).permute(0, 3, 1, 2).float()
    y = F.interpolate(x, size=(nh, nw), mode="bilinear", align_corners=False)
    return y.round().clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).contiguous().numpy()


def write_video(path_noext: str, frames: np.ndarray, fps: float):
    """Write one raw-frame video (``.npy`` + ``.json``) atomically."""
    if frames.dtype != np.uint8 or frames.ndim != 4 or frames.shape[-1] != 3:
        raise ValueError(f"expected uint8 [T,H,W,3], got {frames.dtype} {frames.shape}")
    os.makedirs(os.path.dirname(path_noext), exist_ok=True)
    tmp = path_noext + ".tmp.npy"
    np.save(tmp, np.ascontiguousarray(frames), allow_pickle=False)
    os.replace(tmp, path_noext + ".npy")
    with open(path_noext + ".json", "w") as fh:
        json.dump({"fps": float(fps)}, fh)


def _decode_pyav(path: str) -> Tuple[np.ndarray, float]:  # pragma: no cover - PyAV absent in this image
    import av
    with av.open(path) as c:
        st = c.streams.video[0]
        fps = float(st.average_rate or 30)
        frames = [fr.to_ndarray(format="rgb24") for fr in c.decode(video=0)]
    return np.stack(frames), fps


def _convert_one(job):  # pragma: no cover - needs PyAV
    src, dst_noext, short = job
    if os.path.exists(dst_noext + ".npy"):
        return dst_noext, "skip"
    try:
        frames, fps = _decode_pyav(src)
        if short:
            frames = _resize_short_side(frames, short)
        write_video(dst_noext, frames, fps)
        return dst_noext, "ok"
    except Exception as e:  # corrupt downloads are common in Kinetics: report, continue
        return dst_noext, f"error: {e}"


def list_videos(root: str, exts=VIDEO_EXTENSIONS + FRAME_EXTENSIONS) -> Dict[str, List[Tuple[str, str]]]:
    """split -> [(class_name, path)] in sorted class / file order."""
    out: Dict[str, List[Tuple[str, str]]] = {}
    for split in SPLITS:
        d = os.path.join(root, split)
        if not os.path.isdir(d):
            continue
        items = []
        for cls in sorted(e for e in os.listdir(d) if os.path.isdir(os.path.join(d, e))):
            for f in sorted(os.listdir(os.path.join(d, cls))):
                if os.path.splitext(f)[1].lower() in exts:
                    items.append((cls, os.path.join(d, cls, f)))
        out[split] = items
    return out


def convert(src: str, dst: str, short_side: int = 320, workers: int = 8) -> Dict[str, int]:
    if not pyav_available():
        raise RuntimeError("converting mp4 needs PyAV (`pip install av`) on the conversion host; this ROCm "
                           "image has no video decoder. Convert elsewhere and copy the .npy/.json tree.")
    jobs = []
    for split, items in list_videos(src, VIDEO_EXTENSIONS).items():
        for cls, path in items:
            name = os.path.splitext(os.path.basename(path))[0]
            jobs.append((path, os.path.join(dst, split, cls, name), short_side))
    stats = {"ok": 0, "skip": 0, "error": 0}
    with cf.ProcessPoolExecutor(max_workers=workers) as ex:
        for _, status in ex.map(_convert_one, jobs, chunksize=4):
            stats[status.split(":")[0]] += 1
    return stats


def synthetic(dst: str, classes: int = 4, videos: int = 3, frames: int = 75, height: int = 128, width: int = 170,
              fps: float = 30.0, seed: int = 0) -> int:
    """A small Kinetics-layout raw-frame corpus of random (never all-zero) frames, for tests and demos."""
    rng = np.random.default_rng(seed)
    n = 0
    for split in SPLITS:
        for c in range(classes):
            for v in range(videos if split == "train" else max(1, videos // 2)):
                arr = rng.integers(1, 256, size=(frames, height, width, 3), dtype=np.uint8)
                write_video(os.path.join(dst, split, f"class_{c:03d}", f"vid_{v:04d}"), arr, fps)
                n += 1
    return n


def check(root: str) -> Dict[str, object]:
    """Validate a raw-frame tree: every .npy opens as uint8 [T,H,W,3]; returns counts and class list."""
    report: Dict[str, object] = {}
    bad = []
    for split, items in list_videos(root, FRAME_EXTENSIONS).items():
        classes = sorted({c for c, _ in items})
        for _, p in items:
            try:
                RawFramesVideo(p).close()
            except Exception as e:
                bad.append(f"{p}: {e}")
        report[split] = {"videos": len(items), "classes": len(classes)}
    report["bad"] = bad
    return report


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m pytorchvideo_accelerate_amd.data.prepare")
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("convert")
    c.add_argument("--src", required=True)
    c.add_argument("--dst", required=True)
    c.add_argument("--short_side", type=int, default=320)
    c.add_argument("--workers", type=int, default=8)
    s = sub.add_parser("synthetic")
    s.add_argument("--dst", required=True)
    s.add_argument("--classes", type=int, default=4)
    s.add_argument("--videos", type=int, default=3)
    s.add_argument("--frames", type=int, default=75)
    s.add_argument("--height", type=int, default=128)
    s.add_argument("--width", type=int, default=170)
    k = sub.add_parser("check")
    k.add_argument("--root", required=True)
    a = ap.parse_args(argv)
    if a.cmd == "convert":
        print(json.dumps(convert(a.src, a.dst, a.short_side, a.workers)))
    elif a.cmd == "synthetic":
        print(json.dumps({"written": synthetic(a.dst, a.classes, a.videos, a.frames, a.height, a.width)}))
    else:
        r = check(a.root)
        print(json.dumps(r))
        return 1 if r["bad"] else 0
    return 0


if __name__ == "__main__":
    sys.exit(main())
