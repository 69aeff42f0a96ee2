#!/bin/bash
# streaming pointwise conv kernel: numerics, then the bench step and per-op profile with it in the tuner
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2p
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_pw_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2p/t0.log 2>&1; rc=$?
tail -30 gpurun_out/r2p/t0.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_bnfold_gpu.py tests/test_blocks_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2p/t1.log 2>&1; rc=$?
tail -5 gpurun_out/r2p/t1.log
[ $rc -eq 0 ] || exit 1
PVA_TUNE_LOG=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2p/bench.json 2> gpurun_out/r2p/tune.log || { tail -30 gpurun_out/r2p/tune.log; exit 1; }
cat gpurun_out/r2p/bench.json
timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > gpurun_out/r2p/layers.txt 2> gpurun_out/r2p/layers.err || { tail -20 gpurun_out/r2p/layers.err; exit 1; }
head -1 gpurun_out/r2p/layers.txt
