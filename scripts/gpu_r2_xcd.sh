#!/bin/bash
# XCD-aware wgrad grids: kernel tests, bench, per-op profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2x
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_bnfold_gpu.py -k "wgrad or gram or bnfold" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2x/t0.log 2>&1; rc=$?
tail -4 gpurun_out/r2x/t0.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2x/bench.json 2> gpurun_out/r2x/bench.err || { tail -30 gpurun_out/r2x/bench.err; exit 1; }
cat gpurun_out/r2x/bench.json
PVA_STREAMS=0 timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > gpurun_out/r2x/layers.txt 2> gpurun_out/r2x/layers.err || { tail -20 gpurun_out/r2x/layers.err; exit 1; }
head -1 gpurun_out/r2x/layers.txt
