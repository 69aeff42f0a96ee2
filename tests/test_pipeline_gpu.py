"""GPU input pipeline and end-to-end trainer on the fused gfx950 kernels."""
import json
import os

import numpy as np
import pytest
import torch

from pytorchvideo_accelerate_amd.data.transforms import (ClipParams, GpuClipBatch, pack_pathway_indices,
                                                         reference_transform, sample_params)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ulp(ref: torch.Tensor, mant_bits: int = 7) -> torch.Tensor:
    """One unit in the last place of a ``mant_bits``-bit significand (bf16: 7) at the magnitude of ``ref`` — but never
    below 1e-6: next to zero the fp32 cancellation in x/255 - mean (|x/255| ~ 0.5) already carries ~1e-7 absolute
    error in the reference AND in the kernel (which normalises after interpolating), so a tiny output's last place is
    noise in both."""
    return torch.pow(2.0, torch.floor(torch.log2(ref.abs().clamp_min(2.0 ** -30))) - mant_bits).clamp_min(1e-6)


def test_preprocess_kernel_matches_reference_transform():
    """The fused preprocessing kernel (temporal gather, bilinear short-side resize, crop, flip, normalise, PackPathway)
    is within ONE bf16 ulp of the fp32 reference pipeline at every element."""
    g = torch.Generator().manual_seed(0)
    B, Ts, H, W, T, S = 3, 20, 60, 80, 8, 48
    frames = torch.randint(0, 256, (B, Ts, H, W, 3), generator=g, dtype=torch.uint8)
    params = [sample_params(Ts, H, W, T, S, True, min_scale=50, max_scale=70, generator=g) for _ in range(B)]
    params[1] = ClipParams(params[1].tidx, params[1].rh, params[1].rw, params[1].top, params[1].left, True)
    prep = GpuClipBatch(DEV, T, S, 4)
    slow, fast = prep(frames.to(DEV), params)
    sel = pack_pathway_indices(T, 4)
    for b, p in enumerate(params):
        ref = reference_transform(frames[b], p, S)                       # [3, T, S, S]
        got = fast.t.float().reshape(B, T, S, S, 4)[b].permute(3, 0, 1, 2).cpu()
        assert got[3].abs().max() == 0
        err = (got[:3] - ref).abs()
        assert (err <= _ulp(ref)).all(), float((err / _ulp(ref)).max())
        gs = slow.t.float().reshape(B, len(sel), S, S, 4)[b].permute(3, 0, 1, 2).cpu()
        rs = ref.index_select(1, sel)
        assert ((gs[:3] - rs).abs() <= _ulp(rs)).all()


def test_device_loader_native_reader(tmp_path):
    from pytorchvideo_accelerate_amd.data.kinetics import LabeledVideoPaths, VideoClipDataset
    from pytorchvideo_accelerate_amd.data.loader import DeviceLoader, NativeRawSource, make_host_loader
    rng = np.random.default_rng(0)
    for c in ("a", "b"):
        d = tmp_path / "train" / c
        d.mkdir(parents=True)
        for i in range(3):
            np.save(d / f"v{i}.npy", rng.integers(0, 255, (40, 36 + 4 * i, 48, 3), dtype=np.uint8))
    vids = LabeledVideoPaths.from_directory(str(tmp_path / "train"))
    ds = VideoClipDataset(vids, 1.0, True, num_frames=8, crop_size=32, slowfast_alpha=4, mode="gpu",
                          min_scale=36, max_scale=40)
    src = make_host_loader(ds, 4, num_workers=0, pin_memory=True)
    assert isinstance(src, NativeRawSource) and len(src) == 2
    prep = GpuClipBatch(DEV, 8, 32, 4)
    batches = list(DeviceLoader(src, prep, DEV))
    assert len(batches) == 2 and batches[0]["video"][1].t.shape == (4 * 8 * 32 * 32, 4)
    assert batches[1]["label"].shape == (2,)
    # worker-process DataLoader path gives the same kind of batches
    dl = make_host_loader(ds, 4, num_workers=2, pin_memory=True, native=False)
    b2 = list(DeviceLoader(dl, prep, DEV))
    assert len(b2) == 2 and torch.isfinite(b2[0]["video"][0].t.float()).all()


def test_run_py_fused_gpu(tmp_path):
    import run
    h = run.main(synthetic=True, synthetic_videos=8, synthetic_classes=4, is_slowfast=True, num_frames=8,
                 crop_size=64, batch_size=4, num_workers=0, num_epochs=2, limit_val_batches=1,
                 mixed_precision="bf16", checkpointing_steps="epoch", output_dir=str(tmp_path / "o"),
                 gradient_accumulation_steps=1, lr=0.01, quiet=True, logging_dir=str(tmp_path / "l"))
    assert h["global_step"] == 4 and len(h["accuracy"]) == 2
    assert (tmp_path / "o" / "epoch_1" / "model.safetensors").exists()
    h2 = run.main(synthetic=True, synthetic_videos=8, synthetic_classes=4, is_slowfast=True, num_frames=8,
                  crop_size=64, batch_size=4, num_workers=0, num_epochs=3, limit_val_batches=0,
                  mixed_precision="bf16", resume_from_checkpoint=str(tmp_path / "o" / "epoch_1"),
                  output_dir=str(tmp_path / "o"), gradient_accumulation_steps=1, lr=0.01, quiet=True,
                  logging_dir=str(tmp_path / "l"))
    assert h2["global_step"] == 6


@pytest.mark.parametrize("mp,kernels", [("fp16", "auto"), ("no", "fused"), ("no", "auto"), ("no", "torch")])
def test_run_py_precision_policy(tmp_path, mp, kernels):
    """fp16 = the fp16 fused kernels + dynamic loss scaling (scaler.pt saved/restored); "no" (the reference default, fp32
    math) runs the native fp32 kernels (models/native32.py) unless the fused bf16 kernels or the PyTorch modules are
    asked for explicitly — and the precision that ran is recorded (history / tracker config ``compute_dtype``)."""
    import run
    kw = dict(synthetic=True, synthetic_videos=8, synthetic_classes=4, is_slowfast=True, num_frames=8, crop_size=64,
              batch_size=4, num_workers=0, limit_val_batches=0, mixed_precision=mp, checkpointing_steps="epoch",
              output_dir=str(tmp_path / "o"), gradient_accumulation_steps=2, lr=0.01, quiet=True,
              logging_dir=str(tmp_path / "l"), kernels=kernels)
    h = run.main(num_epochs=1, **kw)
    fused = mp == "fp16" or kernels == "fused"
    assert h["global_step"] == 2
    assert h["backend"] == ("fused" if fused else "torch" if kernels == "torch" else "native32")
    assert h["compute_dtype"] == {"fp16": "fp16", "no": "bf16" if fused else "fp32"}[mp]
    assert (tmp_path / "o" / "epoch_0" / "scaler.pt").exists() == (mp == "fp16")
    if mp == "fp16":
        sd = torch.load(tmp_path / "o" / "epoch_0" / "scaler.pt", weights_only=True)
        assert sd["scale"] == 2.0 ** 16 and sd["_growth_tracker"] == 1   # one clean optimizer step
        h2 = run.main(num_epochs=2, resume_from_checkpoint=str(tmp_path / "o" / "epoch_0"), **kw)
        assert h2["global_step"] == 4


def test_graft_smoke():
    import __graft_entry__ as g
    g.smoke()


def test_preprocess_s2d_layout_matches_dense():
    g = torch.Generator().manual_seed(3)
    B, Ts, H, W, T, S = 2, 12, 40, 50, 8, 32
    frames = torch.randint(0, 256, (B, Ts, H, W, 3), generator=g, dtype=torch.uint8).to(DEV)
    params = [sample_params(Ts, H, W, T, S, True, min_scale=34, max_scale=40, generator=g) for _ in range(B)]
    dense = GpuClipBatch(DEV, T, S, None)(frames, params)[0]
    s2d = GpuClipBatch(DEV, T, S, None, s2d=True)(frames, params)[0]
    from pytorchvideo_accelerate_amd.models.fused import to_s2d
    ref = to_s2d(dense.to_ncthw().float())
    assert s2d.C == 16 and (s2d.H, s2d.W) == (S // 2, S // 2)
    assert torch.equal(s2d.t, ref.t)
