#!/bin/bash
# two-stream executor + asynchronous wgrads + prefetching preprocessing: numerics and bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2pf
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_blocks_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2pf/t0.log 2>&1; rc=$?
tail -5 gpurun_out/r2pf/t0.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2pf/bench.json 2> gpurun_out/r2pf/bench.err || { tail -30 gpurun_out/r2pf/bench.err; exit 1; }
cat gpurun_out/r2pf/bench.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --grad-accum 2 --batch 80 > gpurun_out/r2pf/bench_ga2.json 2> gpurun_out/r2pf/bench_ga2.err || { tail -30 gpurun_out/r2pf/bench_ga2.err; exit 1; }
cat gpurun_out/r2pf/bench_ga2.json
