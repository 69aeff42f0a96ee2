export OUT=r6_last
export BENCHES="--model slow_r50 --frames 8;--precision fp32 --batch 64;--precision fp32 --model slow_r50 --frames 8 --batch 64"
bash scripts/gpu_run.sh benches cfg
