#!/bin/bash
# halo-staged 3x3 conv: numerics, then the headline bench with the tuner log, per-op profile; gradient chaos probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3halo
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_halo_gpu.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
PVA_TUNE_LOG=1 timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
grep -c halo $out/bench.err || true
timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > $out/layers_b160.txt 2> $out/layers.err || { tail -20 $out/layers.err; exit 1; }
head -2 $out/layers_b160.txt
B=4 timeout -k 10 300 python -u scripts/diag_chaos.py > $out/chaos.log 2>&1 || { tail $out/chaos.log; exit 1; }
grep -v MIOpen $out/chaos.log
