#!/bin/bash
# halo-staged weight gradient: numerics, then bench + per-op profile with it in the tuner
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2h
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad_halo" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2h/t0.log 2>&1; rc=$?
tail -25 gpurun_out/r2h/t0.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_blocks_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2h/t1.log 2>&1; rc=$?
tail -5 gpurun_out/r2h/t1.log
[ $rc -eq 0 ] || exit 1
PVA_TUNE_LOG=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2h/bench.json 2> gpurun_out/r2h/tune.log || { tail -30 gpurun_out/r2h/tune.log; exit 1; }
cat gpurun_out/r2h/bench.json
timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > gpurun_out/r2h/layers.txt 2> gpurun_out/r2h/layers.err || { tail -20 gpurun_out/r2h/layers.err; exit 1; }
head -1 gpurun_out/r2h/layers.txt
