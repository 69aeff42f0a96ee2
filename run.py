"""Train SlowFast / Slow ResNet3D action recognition on Kinetics-style data (MI355X-native engine).

Same flags and defaults as the reference ``run.py`` (``main`` kwargs, Fire semantics) plus documented
additions.  Launch like the reference:

    python run.py --is_slowfast --num_frames 32 --sampling_rate 2 --mixed_precision bf16 ...
    python -m pytorchvideo_accelerate_amd.launch --multi_gpu --num_processes 8 run.py ...   # or
    accelerate launch --multi_gpu --num_processes 8 run.py ...      # or
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 run.py ...
"""
from argparse import Namespace

from pytorchvideo_accelerate_amd.engine.trainer import training_function
from pytorchvideo_accelerate_amd.utils.cli import fire_main


def main(
    cpu: bool = False,
    mixed_precision: str = "no",
    checkpointing_steps: str = None,
    resume_from_checkpoint: str = None,
    with_tracking: bool = False,
    logging_dir: str = "pytorchvideo_accelerate_runs",
    output_dir: str = ".",
    log_every: int = 10,
    data_dir: str = "/home/jupyter/data",
    num_frames: int = 8,
    sampling_rate: int = 8,
    frames_per_second: int = 30,
    num_epochs: int = 4,
    pretrained: bool = False,
    lr: float = 0.1,
    momentum: float = 0.9,
    weight_decay: float = 1e-4,
    gradient_accumulation_steps: int = 4,
    num_workers: int = 8,
    batch_size: int = 8,
    limit_train_batches: int = -1,
    limit_val_batches: int = -1,
    is_slowfast: bool = False,
    slowfast_alpha: int = 4,
    freeze_backbone: bool = False,
    pin_memory: bool = False,
    seed: int = 42,
    # ---- additions ----
    crop_size: int = 256,
    model: str = None,
    synthetic: bool = False,
    synthetic_videos: int = 64,
    synthetic_classes: int = 10,
    synthetic_min_frames: int = None,
    kernels: str = "auto",
    reference_val: bool = False,
    pretrained_path: str = None,
    quiet: bool = False,
):
    """Run training of 3D ResNet or SlowFast ResNet for action recognition on Kinetics.

    Reference flags: see reference run.py:328-356.  Additions:
      crop_size          spatial crop (reference fixes 256)
      model              slowfast_r50 | slowfast_r101 | slow_r50 (default from --is_slowfast)
      synthetic          use a synthetic Kinetics-like corpus instead of --data_dir
      synthetic_videos / synthetic_classes   its size
      synthetic_min_frames  vary synthetic video lengths in [this, 300] frames (default: all 300)
      kernels            auto | fused | fp32 | torch  (fused = gfx950 HIP kernels in bf16/fp16; fp32 = gfx950 fp32
                         kernels, the --mixed_precision no default on a GPU; torch = PyTorch modules)
      reference_val      evaluate only one clip per video (reference LimitDataset behaviour)
      pretrained_path    local weights for --pretrained (no network)
    As in the reference, the script flag decides mixed precision (default "no"): the launcher's
    --mixed_precision only reaches programmatic Accelerator(mixed_precision=None) users.
    """
    args = Namespace(**{k: v for k, v in locals().items()})
    return training_function(args)


if __name__ == "__main__":
    fire_main(main)
