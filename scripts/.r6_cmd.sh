export OUT=r6_f32g TESTS="tests/test_native32_gpu.py tests/test_race_gpu.py tests/test_pipeline_gpu.py::test_run_py_precision_policy"
export BENCHES="--precision fp32 --steps 5 --warmup 2;--precision fp32 --batch 64 --steps 5 --warmup 2;PVA_ARMS=f32_pieces=2 --precision fp32 --batch 64 --steps 5 --warmup 2;--precision fp32 --model slow_r50 --frames 8 --batch 64 --steps 5 --warmup 2"
export STOCK="--dtype fp32 --batch 8;--dtype fp32 --batch 32;--dtype fp32 --slow --frames 8 --batch 32;--dtype bf16 --slow --frames 8 --batch 32"
export KSTATS_ARGS="--precision fp32"
bash scripts/gpu_run.sh tests benches kstats stock
