#!/bin/bash
# SlowFast-R50 fine-tuning recipe of the reference (run_slowfast_r50.sh), on the MI355X-native engine.
# --mixed_precision fp16 as in the reference: dynamic loss scaling (GradScaler semantics, scaler.pt) on the
# fused path; the convolutions compute in bf16 MFMA with fp32 master weights (ops/optim.FusedGradScaler).
accelerate launch run.py \
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
