#!/bin/bash
# 1-GPU rehearsal of the multi-rank bench path (2 gloo ranks sharing the device): self-launch, autotune
# agreement, two-stream executor + async wgrads with stage-granular bucket all-reduce
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2d
export TMPDIR=/tmp
PVA_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --batch 16 --steps 4 --warmup 2 > gpurun_out/r2d/bench2.json 2> gpurun_out/r2d/bench2.err || { tail -40 gpurun_out/r2d/bench2.err; exit 1; }
cat gpurun_out/r2d/bench2.json
