#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_optim_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2c/gt1.log 2>&1 || { tail -60 gpurun_out/r2c/gt1.log; exit 1; }
tail -3 gpurun_out/r2c/gt1.log
timeout -k 10 600 python -u -m pytest tests/test_fullshape_gpu.py -x -v --timeout 500 --timeout-method thread > gpurun_out/r2c/gt2.log 2>&1 || { tail -60 gpurun_out/r2c/gt2.log; exit 1; }
tail -8 gpurun_out/r2c/gt2.log
