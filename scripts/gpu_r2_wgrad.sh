#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2d
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k wgrad --timeout 200 --timeout-method thread > gpurun_out/r2d/gt.log 2>&1 || { tail -60 gpurun_out/r2d/gt.log; exit 1; }
tail -2 gpurun_out/r2d/gt.log
PVA_TUNE_LOG=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2d/bench.json 2> gpurun_out/r2d/tune.log || { tail -30 gpurun_out/r2d/tune.log; exit 1; }
cat gpurun_out/r2d/bench.json
