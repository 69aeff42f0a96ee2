#!/bin/bash
# pointwise kernel specialised per epilogue operand stream: numerics, bandwidth probe, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r2ops
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pw_gpu.py tests/test_blocks_gpu.py > $D/tests.txt 2>&1 || { tail -30 $D/tests.txt; exit 1; }
tail -2 $D/tests.txt
timeout -k 10 200 python -u scripts/pw_probe.py > $D/probe.txt 2>&1 || { tail -20 $D/probe.txt; exit 1; }
grep us $D/probe.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $D/bench.json 2> $D/bench.err || { tail -30 $D/bench.err; exit 1; }
python -c 'import json,sys; d=json.load(open(sys.argv[1])); print("bench", d["value"], d["ms_per_step"])' $D/bench.json
