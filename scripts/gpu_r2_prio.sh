#!/bin/bash
# fast-pathway stream priority sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2pr
export TMPDIR=/tmp
for pr in -1 0; do
  PVA_SIDE_PRIORITY=$pr timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2pr/b$pr.json 2> gpurun_out/r2pr/e$pr.log || { tail -20 gpurun_out/r2pr/e$pr.log; exit 1; }
  echo "prio $pr $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"])' gpurun_out/r2pr/b$pr.json)"
done
