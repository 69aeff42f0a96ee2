#!/bin/bash
# batch-size sweep at the headline config and the other SURVEY model configs on the round-3 kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3cfg
mkdir -p $out
export TMPDIR=/tmp
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }
  echo "$name $(python -c "import json,sys; d=json.load(open('$out/$name.json')); print(d['value'], d['ms_per_step'], d['config']['peak_mem_gb'])")"
}
run b192 --batch 192 --steps 12 --warmup 4
run b224 --batch 224 --steps 12 --warmup 4
run b256 --batch 256 --steps 12 --warmup 4
run r101_256_b48 --depth 101 --crop 256 --batch 48 --steps 12 --warmup 4
run r50_64x2_gas4_b24 --frames 64 --batch 24 --grad-accum 4 --steps 6 --warmup 2
