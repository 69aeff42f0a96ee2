"""CLI flag parity (Fire semantics) and model architecture parity (§2.3)."""
import inspect

import pytest
import torch

import run
from pytorchvideo_accelerate_amd.engine.trainer import build_model, parse_checkpointing_steps
from pytorchvideo_accelerate_amd.models import reference as R
from pytorchvideo_accelerate_amd.utils.cli import parse_fire_args

REFERENCE_DEFAULTS = {
    "cpu": False, "mixed_precision": "no", "checkpointing_steps": None, "resume_from_checkpoint": None,
    "with_tracking": False, "logging_dir": "pytorchvideo_accelerate_runs", "output_dir": ".", "log_every": 10,
    "data_dir": "/home/jupyter/data", "num_frames": 8, "sampling_rate": 8, "frames_per_second": 30,
    "num_epochs": 4, "pretrained": False, "lr": 0.1, "momentum": 0.9, "weight_decay": 1e-4,
    "gradient_accumulation_steps": 4, "num_workers": 8, "batch_size": 8, "limit_train_batches": -1,
    "limit_val_batches": -1, "is_slowfast": False, "slowfast_alpha": 4, "freeze_backbone": False,
    "pin_memory": False, "seed": 42,
}


def test_all_reference_flags_and_defaults():
    sig = inspect.signature(run.main)
    for k, v in REFERENCE_DEFAULTS.items():
        assert k in sig.parameters, k
        assert sig.parameters[k].default == v, k
    assert len(REFERENCE_DEFAULTS) == 27


def test_fire_semantics():
    a = parse_fire_args(run.main, ["--is_slowfast", "--num_frames", "32", "--lr=0.05", "--checkpointing_steps",
                                   "1000", "--mixed-precision", "bf16", "--nopin_memory", "--data_dir", "/x/y"])
    assert a["is_slowfast"] is True and a["num_frames"] == 32 and a["lr"] == 0.05
    assert a["checkpointing_steps"] == 1000 and isinstance(a["checkpointing_steps"], int)  # Fire -> int (R7a)
    assert a["mixed_precision"] == "bf16" and a["pin_memory"] is False and a["data_dir"] == "/x/y"
    b = parse_fire_args(run.main, ["--checkpointing_steps", "epoch", "--with_tracking", "True"])
    assert b["checkpointing_steps"] == "epoch" and b["with_tracking"] is True
    with pytest.raises(SystemExit):
        parse_fire_args(run.main, ["--not_a_flag", "1"])


def test_checkpointing_steps_parsing_fixes_fire_int_bug():
    assert parse_checkpointing_steps(1000) == 1000      # reference silently returned None here
    assert parse_checkpointing_steps("1000") == 1000
    assert parse_checkpointing_steps("epoch") == "epoch"
    assert parse_checkpointing_steps(None) is None
    with pytest.raises(ValueError):
        parse_checkpointing_steps("often")


def test_param_counts_match_model_zoo():
    assert R.count_params(R.slowfast_r50(400)) == 34_566_488
    assert R.count_params(R.slow_r50(400)) == 32_454_096


def test_state_dict_keys_follow_pytorchvideo_tree():
    keys = list(R.slowfast_r50(10).state_dict().keys())
    for k in ["blocks.0.multipathway_blocks.0.conv.weight", "blocks.0.multipathway_fusion.conv_fast_to_slow.weight",
              "blocks.1.multipathway_blocks.0.res_blocks.0.branch1_conv.weight",
              "blocks.1.multipathway_blocks.0.res_blocks.0.branch2.conv_a.weight",
              "blocks.4.multipathway_blocks.1.res_blocks.2.branch2.norm_c.running_var",
              "blocks.6.proj.weight", "blocks.6.proj.bias"]:
        assert k in keys, k
    keys = list(R.slow_r50(10).state_dict().keys())
    assert "blocks.0.conv.weight" in keys and "blocks.5.proj.weight" in keys


def test_head_replacement_and_freeze():
    class A:
        is_slowfast, model, crop_size, num_frames, slowfast_alpha = True, None, 224, 32, 4
        pretrained, freeze_backbone = False, True
    m = build_model(A, 700)
    assert m.blocks[-1].proj.out_features == 700 and m.blocks[-1].proj.in_features == 2304
    assert m.blocks[-1].pool is None
    assert not any(p.requires_grad for p in m.blocks[:-1].parameters())
    assert all(p.requires_grad for p in m.blocks[-1].parameters())
    A.is_slowfast, A.freeze_backbone = False, False
    m2 = build_model(A, 5)
    assert tuple(m2.blocks[-1].pool.kernel_size) == (1, 7, 7) and m2.blocks[-1].proj.in_features == 2048


def test_poolconcat_256_crop_overlapping_windows_and_64_frame_fallback():
    pool = R.PoolConcatPathway(((8, 7, 7), (32, 7, 7)))
    xs = [torch.randn(1, 4, 8, 8, 8), torch.randn(1, 2, 32, 8, 8)]
    y = pool(xs)
    assert y.shape == (1, 6, 1, 2, 2)  # exact overlapping 7x7 windows at 256^2
    torch.testing.assert_close(y[:, :4, 0, 0, 0], xs[0][:, :, :, :7, :7].mean((2, 3, 4)))
    xs64 = [torch.randn(1, 4, 16, 7, 7), torch.randn(1, 2, 64, 7, 7)]
    y64 = pool(xs64)  # the stock head crashes here; we fall back to a global average
    assert y64.shape == (1, 6, 1, 1, 1)


def test_slowfast_forward_cpu_shape():
    m = R.create_slowfast(50, 7, head_pool_kernel_sizes=((2, 2, 2), (8, 2, 2))).eval()
    with torch.no_grad():
        out = m([torch.randn(1, 3, 2, 64, 64), torch.randn(1, 3, 8, 64, 64)])
    assert out.shape == (1, 7)
