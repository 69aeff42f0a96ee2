#!/bin/bash
# two-level BN finalize: kernel tests, fused-executor tests, bench + per-op profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3fin
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_pool_kernels_gpu.py tests/test_fused_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
PVA_TUNE_LOG=1 timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 python -u scripts/layer_profile.py --batch 160 --steps 2 > $out/layers_b160.txt 2> $out/layers.err || { tail -20 $out/layers.err; exit 1; }
head -2 $out/layers_b160.txt
