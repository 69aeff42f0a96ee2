#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bnfold_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2e/gt0.log 2>&1; rc=$?
tail -30 gpurun_out/r2e/gt0.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_blocks_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2e/gt1.log 2>&1; rc=$?
tail -30 gpurun_out/r2e/gt1.log
[ $rc -eq 0 ] || exit 1
PVA_TUNE_LOG=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2e/bench.json 2> gpurun_out/r2e/tune.log || { tail -30 gpurun_out/r2e/tune.log; exit 1; }
cat gpurun_out/r2e/bench.json
