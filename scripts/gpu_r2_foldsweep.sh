#!/bin/bash
# bench step with the conv_c BN fold enabled down to fold_min_c channels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2s
export TMPDIR=/tmp
for c in 8 16 32; do
  PVA_BN_FOLD_MIN_C=$c timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2s/bench_$c.json 2> gpurun_out/r2s/err_$c.log || { tail -20 gpurun_out/r2s/err_$c.log; exit 1; }
  echo "fold_min_c=$c $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"])' gpurun_out/r2s/bench_$c.json)"
done
