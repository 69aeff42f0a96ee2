export OUT=r6_f32v3 TESTS=tests/test_native32_gpu.py
export BENCHES="--precision fp32 --batch 64 --steps 6 --warmup 2;--precision fp32 --model slow_r50 --frames 8 --batch 64 --steps 6 --warmup 2"
bash scripts/gpu_run.sh tests benches
