#!/bin/bash
# SlowFast-R50 fine-tuning recipe of the reference (run_slowfast_r50.sh), on the MI355X-native engine.
# The launcher (pytorchvideo_accelerate_amd/launch.py, accelerate-launch compatible) starts one rank per visible
# GPU when no accelerate config file exists, like the reference's bare `accelerate launch`.
# --mixed_precision fp16 as in the reference: the convolutions run fp16 MFMA kernels with fp32 master weights and
# dynamic loss scaling (GradScaler semantics, scaler.pt; ops/optim.FusedGradScaler).
python -m pytorchvideo_accelerate_amd.launch run.py \
    --output_dir outputs \
    --batch_size 8 \
    --num_workers 8 \
    --gradient_accumulation_steps 4 \
    --checkpointing_steps epoch \
    --mixed_precision fp16 \
    --with_tracking \
    --num_frames 32 \
    --sampling_rate 2 \
    --is_slowfast \
    --pin_memory "$@"
