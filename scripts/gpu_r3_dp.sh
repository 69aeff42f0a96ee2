#!/bin/bash
# multi-rank fused DP tests + precision policy + direct-kernel bit change
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3dp
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread -m gpu tests/test_dp_fused_gpu.py tests/test_pipeline_gpu.py tests/test_conv_direct_gpu.py tests/test_graph_gpu.py > $out/gt.log 2>&1
rc=$?
tail -30 $out/gt.log
exit $rc
