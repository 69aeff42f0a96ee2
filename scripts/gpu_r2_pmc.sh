#!/bin/bash
# BN/pool kernel unit tests, then PMC counters of one bench step at B=64
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2m
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bn_pool_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2m/t0.log 2>&1; rc=$?
tail -25 gpurun_out/r2m/t0.log
[ $rc -eq 0 ] || exit 1
PMC_OUT=r2m/pmc BATCH=64 bash scripts/gpu_pmc_step.sh
