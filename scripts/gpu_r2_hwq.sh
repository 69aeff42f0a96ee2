#!/bin/bash
# hardware queue count A/B (the step uses 5 HIP streams: main, fast pathway, 2 wgrad, preprocessing)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2q
mkdir -p $out
for q in ${QS:-4 8 16 4 8}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $out/q$q.json 2> $out/q$q.err || { tail -10 $out/q$q.err; exit 1; }
  echo "hwq=$q $(cut -c100-180 $out/q$q.json)"
done
