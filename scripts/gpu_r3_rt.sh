#!/bin/bash
# row-table wgrad kernel: kernel tests vs fp32 PyTorch, micro-benchmark vs the generic kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3rt
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "rowtable or wgrad" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 500 python -u scripts/wgrad_bench.py 2>&1 | grep -v amdgpu.ids | tee $out/wgrad_bench.txt
