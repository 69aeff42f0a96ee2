#!/bin/bash
# HIP-graph step: GPU tests, then eager vs graph bench at the headline batch and at small per-GPU batches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2g
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_head_gpu.py tests/test_fused_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/gt.log 2>&1 || { tail -40 $out/gt.log; exit 1; }
tail -1 $out/gt.log
for B in 16 160; do
  for G in 0 1; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch $B --graph $G > $out/b${B}_g$G.json 2> $out/b${B}_g$G.err || { tail -20 $out/b${B}_g$G.err; exit 1; }
    echo "B=$B graph=$G $(cut -c100-200 $out/b${B}_g$G.json)"
  done
done
