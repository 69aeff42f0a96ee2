#!/bin/bash
# non-temporal output stores in the pointwise kernel: bandwidth probe A/B, then bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2nt
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/pw_probe.py > gpurun_out/r2nt/probe0.txt 2>&1 || { tail -20 gpurun_out/r2nt/probe0.txt; exit 1; }
PVA_PW_NT=1 timeout -k 10 200 python -u scripts/pw_probe.py > gpurun_out/r2nt/probe1.txt 2>&1 || { tail -20 gpurun_out/r2nt/probe1.txt; exit 1; }
paste gpurun_out/r2nt/probe0.txt gpurun_out/r2nt/probe1.txt | grep us
PVA_PW_NT=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2nt/bench_nt.json 2> gpurun_out/r2nt/bench_nt.err || { tail -30 gpurun_out/r2nt/bench_nt.err; exit 1; }
python -c 'import json,sys; d=json.load(open(sys.argv[1])); print("nt", d["value"], d["ms_per_step"])' gpurun_out/r2nt/bench_nt.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2nt/bench.json 2> gpurun_out/r2nt/bench.err || { tail -30 gpurun_out/r2nt/bench.err; exit 1; }
python -c 'import json,sys; d=json.load(open(sys.argv[1])); print("default", d["value"], d["ms_per_step"])' gpurun_out/r2nt/bench.json
