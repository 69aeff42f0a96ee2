#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2b/gt.log 2>&1 || { tail -60 gpurun_out/r2b/gt.log; exit 1; }
tail -3 gpurun_out/r2b/gt.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2b/smoke.log 2>&1 || { tail -30 gpurun_out/r2b/smoke.log; exit 1; }
tail -2 gpurun_out/r2b/smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2b/bench.json 2> gpurun_out/r2b/bench.err || { tail -30 gpurun_out/r2b/bench.err; exit 1; }
cat gpurun_out/r2b/bench.json
