#!/bin/bash
# A/B of the conv_c BN-fold threshold on the current kernels (fast pathway res2 cin=8, res3 cin=16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2fc
mkdir -p $out
for C in 32 16 8; do
  PVA_BN_FOLD_MIN_C=$C timeout -k 10 300 python bench.py --steps 12 --warmup 4 > $out/c$C.json 2> $out/c$C.err || { tail -5 $out/c$C.err; exit 1; }
  echo "min_c=$C $(cut -c1-150 $out/c$C.json)"
done
