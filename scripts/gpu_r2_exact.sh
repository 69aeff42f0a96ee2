#!/bin/bash
# exact-statistics narrow folds: determinism diag, block/fused tests with every unit folded, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2x
mkdir -p $out
export TMPDIR=/tmp
PVA_BN_FOLD_MIN_C=8 timeout -k 10 300 python scripts/diag_ms_fold.py > $out/diag.txt 2>&1 || { tail -20 $out/diag.txt; exit 1; }
grep stream $out/diag.txt
PVA_BN_FOLD_MIN_C=8 timeout -k 10 600 python -u -m pytest tests/test_blocks_gpu.py tests/test_fused_gpu.py tests/test_fullshape_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/gt.log 2>&1 || { tail -30 $out/gt.log; exit 1; }
tail -1 $out/gt.log
for C in 8 32; do
  PVA_BN_FOLD_MIN_C=$C timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $out/c$C.json 2> $out/c$C.err || { tail -5 $out/c$C.err; exit 1; }
  echo "min_c=$C $(cut -c100-175 $out/c$C.json)"
done
