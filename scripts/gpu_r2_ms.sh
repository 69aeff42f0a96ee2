#!/bin/bash
# two-stream (slow / fast pathway) execution: numerics, then bench with and without it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2s2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_blocks_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2s2/t0.log 2>&1; rc=$?
tail -5 gpurun_out/r2s2/t0.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2s2/bench_ms.json 2> gpurun_out/r2s2/bench_ms.err || { tail -30 gpurun_out/r2s2/bench_ms.err; exit 1; }
cat gpurun_out/r2s2/bench_ms.json
PVA_STREAMS=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2s2/bench_1s.json 2> gpurun_out/r2s2/bench_1s.err || { tail -30 gpurun_out/r2s2/bench_1s.err; exit 1; }
cat gpurun_out/r2s2/bench_1s.json
