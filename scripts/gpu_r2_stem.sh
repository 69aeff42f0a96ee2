#!/bin/bash
# fused stem pool/BN backward: numerics, block/model parity, bench + per-op profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2t
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bn_pool_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2t/t0.log 2>&1; rc=$?
tail -15 gpurun_out/r2t/t0.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u -m pytest tests/test_blocks_gpu.py tests/test_fused_gpu.py tests/test_fullshape_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2t/t1.log 2>&1; rc=$?
tail -5 gpurun_out/r2t/t1.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2t/bench.json 2> gpurun_out/r2t/bench.err || { tail -30 gpurun_out/r2t/bench.err; exit 1; }
cat gpurun_out/r2t/bench.json
timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > gpurun_out/r2t/layers.txt 2> gpurun_out/r2t/layers.err || { tail -20 gpurun_out/r2t/layers.err; exit 1; }
head -1 gpurun_out/r2t/layers.txt
