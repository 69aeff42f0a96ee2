#!/bin/bash
# Round-2 first GPU pass: GPU tests, headline bench, steady-state kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2a/gt.log 2>&1 || { tail -40 gpurun_out/r2a/gt.log; exit 1; }
tail -3 gpurun_out/r2a/gt.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err || { tail -30 gpurun_out/r2a/bench.err; exit 1; }
cat gpurun_out/r2a/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r2a/prof -o k --output-format csv -- python3 bench.py --steps 3 --warmup 2 --batch 96 > gpurun_out/r2a/prof.log 2>&1 || { tail -20 gpurun_out/r2a/prof.log; exit 1; }
f=$(find gpurun_out/r2a/prof -name '*kernel_trace.csv' | head -1)
python scripts/steady_state_kernels.py "$f" --steps 2 --top 60 > gpurun_out/r2a/kernels_steady_state.txt
head -50 gpurun_out/r2a/kernels_steady_state.txt
