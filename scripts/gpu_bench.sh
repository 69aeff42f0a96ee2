#!/bin/bash
# 1-GPU bench at a few batch sizes + rocprofv3 kernel summary of a short run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in ${BATCHES:-8 16}; do
  timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 3 --batch $b > gpurun_out/bench_b$b.json 2> gpurun_out/bench_b$b.err || { tail -30 gpurun_out/bench_b$b.err; exit 1; }
  cat gpurun_out/bench_b$b.json
done
if [ -n "$PROFILE" ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ours -o ours --output-format csv -- python3 bench.py --steps 3 --warmup 2 --batch ${PROFILE} > gpurun_out/prof_ours.log 2>&1 || { tail -20 gpurun_out/prof_ours.log; exit 1; }
fi
