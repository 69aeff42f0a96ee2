#!/bin/bash
# stream configuration A/B on the final kernels: default, fast-pathway stream high priority, single stream
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2sab
mkdir -p $out
for v in "X=0" "PVA_SIDE_PRIORITY=-1" "PVA_STREAMS=0" "X=1"; do
  env $v timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $out/b.json 2> $out/b.err || { tail -10 $out/b.err; exit 1; }
  echo "$v $(cut -c100-180 $out/b.json)"
done
