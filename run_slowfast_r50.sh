#!/bin/bash
# SlowFast-R50 fine-tuning recipe of the reference (run_slowfast_r50.sh), on the MI355X-native engine.
# fp16 requests run the bf16 gfx950 kernels (bf16 has fp32 range; no loss scaling needed).
accelerate launch run.py \
    --output_dir outputs \
    --batch_size 8 \
    --num_workers 8 \
    --gradient_accumulation_steps 4 \
    --checkpointing_steps epoch \
    --mixed_precision bf16 \
    --with_tracking \
    --num_frames 32 \
    --sampling_rate 2 \
    --is_slowfast \
    --pin_memory "$@"
