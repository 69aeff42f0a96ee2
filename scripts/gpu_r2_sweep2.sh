#!/bin/bash
# batch sweep of the current state + hipBLASLt reference GEMMs at the conv shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2s
mkdir -p $out
for B in 192 224; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch $B > $out/b$B.json 2> $out/b$B.err || { tail -5 $out/b$B.err; exit 1; }
  cut -c1-160 $out/b$B.json
done
timeout -k 10 300 python scripts/gemm_probe.py > $out/gemm_probe.txt 2>&1 || { tail -5 $out/gemm_probe.txt; exit 1; }
cat $out/gemm_probe.txt
