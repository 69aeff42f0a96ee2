#!/bin/bash
# BN-fold coverage A/B at the headline config: default (slow pathway, conv_c inputs >= 32 channels) vs folding the
# fast pathway's narrow units too (exact statistics pass, models/fused.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3fold
mkdir -p $out
export TMPDIR=/tmp
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }
  echo "$name $(python -c "import json,sys; d=json.load(open('$out/$name.json')); print(d['value'], d['ms_per_step'], d['config']['final_loss'])")"
}
run base PVA_NOOP=1
run fold16 PVA_BN_FOLD_MIN_C=16
run fold8 PVA_BN_FOLD_MIN_C=8
run base2 PVA_NOOP=1
