#!/bin/bash
# Run GPU test files given as args (default: all gpu tests).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest ${@:-tests} -x -q -m gpu > gpurun_out/gt.log 2>&1
rc=$?
tail -40 gpurun_out/gt.log
exit $rc
