#!/bin/bash
# Batch-size sweep + the secondary BASELINE.json configs on one GPU.  Output: gpurun_out/sweep/*.json
set -o pipefail
mkdir -p gpurun_out/sweep
run() {  # name, args...
  local n=$1; shift
  echo "== $n $*"
  timeout -k 10 420 python bench.py --steps 12 --warmup 2 "$@" > gpurun_out/sweep/$n.json 2> gpurun_out/sweep/$n.err
  local rc=$?
  cat gpurun_out/sweep/$n.json
  return $rc
}
run b96 --batch 96 && run b128 --batch 128 && run b160 --batch 160 && run b192 --batch 192 &&
run r101_256_b48 --depth 101 --crop 256 --batch 48 &&
run r50_64x2_gas4_b24 --frames 64 --src-frames 128 --batch 24 --grad-accum 4
