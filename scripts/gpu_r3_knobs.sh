#!/bin/bash
# kernel-family A/B under the real (two-stream) schedule: the autotuner picks per geometry in isolation (first
# step, one stream); these runs drop one candidate family at a time and measure the whole step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3knobs
mkdir -p $out
export TMPDIR=/tmp
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }
  echo "$name $(python -c "import json,sys; d=json.load(open('$out/$name.json')); print(d['value'], d['ms_per_step'])")"
}
run base PVA_NOOP=1
run no_dma PVA_CONV_DMA=0
run no_direct PVA_CONV_DIRECT=0
run no_fold1 PVA_BN_FOLD1=0
run base2 PVA_NOOP=1
