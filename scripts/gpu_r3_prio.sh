#!/bin/bash
# stream-priority A/B at the headline config: the critical path is the slow-pathway (main) stream, always busy
# (profiles/r3_re); the fast-pathway and weight-gradient side streams compete with it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3prio
mkdir -p $out
export TMPDIR=/tmp
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 1; }
  echo "$name $(python -c "import json,sys; d=json.load(open('$out/$name.json')); print(d['value'], d['ms_per_step'])")"
}
run base PVA_NOOP=1
run main_hi PVA_MAIN_PRIORITY=-1
run main_hi_side_hi PVA_MAIN_PRIORITY=-1 PVA_SIDE_PRIORITY=-1
run wgrad_lo PVA_WGRAD_PRIORITY=1
run base2 PVA_NOOP=1
