"""End-to-end trainer on CPU (BASELINE config 1 plumbing at toy size): checkpoint/resume semantics."""
import os

import run


def _args(tmp, **kw):
    a = dict(cpu=True, synthetic=True, synthetic_videos=8, synthetic_classes=3, num_frames=8, crop_size=64,
             batch_size=2, num_workers=0, num_epochs=2, limit_val_batches=0, output_dir=str(tmp / "out"),
             gradient_accumulation_steps=2, quiet=True, logging_dir=str(tmp / "logs"))
    a.update(kw)
    return a


def test_step_checkpoints_and_resume(tmp_path):
    h = run.main(**_args(tmp_path, checkpointing_steps=3, with_tracking=True, limit_train_batches=-1))
    assert h["global_step"] == 8  # 2 epochs x 4 batches (8 videos / batch 2)
    out = tmp_path / "out"
    assert (out / "step_3").is_dir() and (out / "step_6").is_dir()
    assert os.path.exists(tmp_path / "logs" / (str(tmp_path / "logs").replace(".", "").replace("/", "")) /
                          "metrics.jsonl")
    # resume mid-epoch-1 from step_6: continues at global step 6 (reference restarted at 0)
    h2 = run.main(**_args(tmp_path, resume_from_checkpoint=str(out / "step_6"), checkpointing_steps="epoch"))
    assert h2["global_step"] == 8
    assert (out / "epoch_1").is_dir() and not (out / "epoch_0").is_dir()
    # "latest" resolves to the newest checkpoint directory
    h3 = run.main(**_args(tmp_path, resume_from_checkpoint="latest", num_epochs=2))
    assert h3["global_step"] == 8


def test_slow_r50_epoch_checkpoint_and_final(tmp_path):
    h = run.main(**_args(tmp_path, num_epochs=1, limit_train_batches=0, freeze_backbone=True))
    assert h["final_dir"].endswith("final") and os.path.exists(os.path.join(h["final_dir"], "model.safetensors"))


def test_progress_bar_on_main_process(tmp_path, capsys):
    """reference run.py:233-288: tqdm over num_epochs * len(train_loader), "Epoch: e" / "Val Epoch: e"."""
    run.main(**_args(tmp_path, num_epochs=1, limit_train_batches=-1, quiet=False))
    err = capsys.readouterr().err
    assert "Epoch: 0" in err and "Val Epoch: 0" in err
    assert "4/4" in err   # 8 videos / batch 2 = 4 steps, all updated


def test_progress_fallback_bar():
    import io
    from pytorchvideo_accelerate_amd.utils.progress import _FallbackBar
    f = io.StringIO()
    b = _FallbackBar(3, file=f, mininterval=0.0)
    b.set_description_str("Epoch: 0")
    for _ in range(3):
        b.update(1)
    b.close()
    assert "Epoch: 0" in f.getvalue() and "3/3" in f.getvalue()
