#!/bin/bash
# Round-2 re-entry checkpoint: GPU test suite, headline bench, steady-state kernel trace, per-op profile (B=160).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUTD:-r2e}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gt.log 2>&1 || { tail -40 $out/gt.log; exit 1; }
tail -3 $out/gt.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o k --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name '*kernel_trace.csv' | head -1)
python scripts/steady_state_kernels.py "$f" --steps 2 --top 60 > $out/kernels_steady_state.txt
head -30 $out/kernels_steady_state.txt
timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > $out/layers_b160.txt 2> $out/layers.err || { tail -20 $out/layers.err; exit 1; }
tail -25 $out/layers_b160.txt
