#!/bin/bash
# bandwidth probe of the pointwise kernel only
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r2probe
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/pw_probe.py > $D/probe.txt 2>&1 || { tail -20 $D/probe.txt; exit 1; }
grep us $D/probe.txt
