#!/bin/bash
# Iteration check: targeted GPU tests (args), headline bench, per-op profile at the bench batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-r2i}
mkdir -p $out
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q -m gpu --timeout 300 --timeout-method thread > $out/gt.log 2>&1 || { tail -40 $out/gt.log; exit 1; }
  tail -3 $out/gt.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
if [ -z "$NOLAYERS" ]; then
  timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > $out/layers_b160.txt 2> $out/layers.err || { tail -20 $out/layers.err; exit 1; }
  grep -E "^#|stem|b0\.|head" $out/layers_b160.txt | head -40
fi
