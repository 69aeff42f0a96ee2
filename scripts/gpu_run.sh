#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment gpu_r*_*.sh scripts, which live in git history).
#   scripts/gpu_run.sh TASK [TASK ...]      every task writes under gpurun_out/$OUT (default: run)
# tasks (run in the order given; the first failure ends the call — no GPU step after a failed one):
#   smoke    __graft_entry__.smoke()
#   tests    pytest -m gpu over $TESTS (default: tests), per-test timeout
#   bench    bench.py $BENCH_ARGS (tuner log in bench.err)          host   bench.py --source host $BENCH_ARGS
#   fp16     bench.py --precision fp16 $BENCH_ARGS
#   ab       bench.py under each setting of $AB (";"-separated env assignments, e.g. AB="PVA_X=0;PVA_X=1")
#   sweep    bench.py $BENCH_ARGS at every batch size of $SWEEP (memory / throughput sweep; stops at the first OOM)
#   layers   serialised per-op profile at B=$BATCH (default 160) + roofline table
#   trace    rocprofv3 kernel trace of 3 steps -> steady-state kernel table
#   pmc      rocprofv3 PMC passes (one run each) over a bench step at B=$BATCH -> per-kernel summary
#            ($PMC_ARGS replaces "--batch $BATCH", $PMC_TAG the summary's suffix, e.g. the fp32 path)
#   cfg      non-headline configs: bench + serialised per-op profile + roofline for R101 32x2x256 (B=160) and
#            R50 64x2x224 (B=112)
#   runpy    the reference CLI (run.py) at the headline shape on a synthetic corpus
#   kstats   rocprofv3 --stats of bench.py $KSTATS_ARGS: per-kernel totals (kernel_stats.csv + top-25 table)
#   losstraj the bench recipe through the bf16 and fp32 executors side by side (diag_loss_trajectory.py, $LT_ARGS)
#   benches  bench.py once per ";"-separated $BENCHES argument set
#   stock    stock PyTorch eager baselines (scripts/baseline_torch.py) for each ";"-separated $STOCK argument set
#   lab      tools/gemm_lab.hip: big-tile GEMM main loop at $LAB_SHAPES ("M,N,K ..."), cold and L2-hot A operand,
#            plus one PMC pass per shape (MFMA busy, waits, L2 hits)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-run}
mkdir -p "$out"
B=${BATCH:-160}

fail() { tail -${2:-30} "$1"; exit 1; }

t_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || fail $out/smoke.log; tail -1 $out/smoke.log; }
t_tests() {
  # -s: the long tests print per-step progress, so a slow test is visibly alive (the runner kills silent commands)
  timeout -k 10 1500 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || fail $out/tests.log 60
  grep -E "passed|failed" $out/tests.log | tail -2
}
t_bench() { PVA_TUNE_LOG=1 timeout -k 10 400 python bench.py $BENCH_ARGS > $out/bench.json 2> $out/bench.err || fail $out/bench.err; cat $out/bench.json; }
t_host() { timeout -k 10 400 python bench.py --source host $BENCH_ARGS > $out/bench_host.json 2> $out/bench_host.err || fail $out/bench_host.err; cat $out/bench_host.json; }
t_fp16() { PVA_TUNE_LOG=1 timeout -k 10 400 python bench.py --precision fp16 $BENCH_ARGS > $out/bench_fp16.json 2> $out/bench_fp16.err || fail $out/bench_fp16.err; cat $out/bench_fp16.json; }
t_ab() {
  local i=0
  IFS=';' read -ra arms <<< "$AB"
  for arm in "${arms[@]}"; do
    i=$((i+1))
    env PVA_TUNE_LOG=1 $arm timeout -k 10 400 python bench.py $BENCH_ARGS > $out/ab$i.json 2> $out/ab$i.err || fail $out/ab$i.err
    echo "$arm: $(cat $out/ab$i.json)"
  done
}
t_sweep() {
  for b in $SWEEP; do
    timeout -k 10 500 python bench.py --batch $b --steps ${STEPS:-8} --warmup 2 $BENCH_ARGS > $out/sweep_b$b.json 2> $out/sweep_b$b.err || { tail -3 $out/sweep_b$b.err; break; }
    echo "B=$b $(python3 -c "import json; d=json.load(open('$out/sweep_b$b.json')); print(d['value'], 'clips/s', d['ms_per_step'], 'ms', d['config'].get('peak_mem_gb'), 'GB')")"
  done
}
t_layers() {
  timeout -k 10 400 python -u scripts/layer_profile.py --batch $B --steps 2 > $out/layers_b$B.txt 2> $out/layers.err || fail $out/layers.err
  head -1 $out/layers_b$B.txt
  python scripts/layer_roofline.py $out/layers_b$B.txt --batch $B > $out/layers_roofline_b$B.txt && grep -A 12 "# totals" $out/layers_roofline_b$B.txt
}
t_trace() {
  timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $out/prof -o step -- python3 bench.py --steps 3 --warmup 3 $BENCH_ARGS > $out/prof.log 2>&1 || fail $out/prof.log
  local f
  f=$(ls $out/prof/*/step_kernel_trace.csv $out/prof/step_kernel_trace.csv 2>/dev/null | head -1)
  python scripts/steady_state_kernels.py "$f" --steps 2 > $out/kernels_steady_state.txt && head -3 $out/kernels_steady_state.txt
  rm -f "$f"
}
t_pmc() {
  local P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  local i=0 tag=${PMC_TAG:-b$B}
  for P in "$P1" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 420 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $out/pmc/p$i -o p -- python3 bench.py --steps 2 --warmup 1 ${PMC_ARGS:---batch $B} > $out/pmc_${tag}_p$i.log 2>&1 || fail $out/pmc_${tag}_p$i.log 5
  done
  # raw per-dispatch CSVs are large (gpurun copies back at most 64 MiB): keep the summary only
  python3 scripts/pmc_step_summary.py $out/pmc > $out/pmc_summary_$tag.txt && rm -rf $out/pmc && head -30 $out/pmc_summary_$tag.txt
}
t_cfg() {
  local spec tag args
  for spec in "r101:--depth 101 --crop 256:160" "f64:--frames 64:112"; do
    IFS=':' read -r tag args b <<< "$spec"
    timeout -k 10 500 python bench.py --batch $b --steps 10 --warmup 3 $args > $out/cfg_$tag.json 2> $out/cfg_$tag.err || fail $out/cfg_$tag.err
    cat $out/cfg_$tag.json
    timeout -k 10 500 python -u scripts/layer_profile.py --batch $b --steps 2 $args > $out/cfg_${tag}_layers.txt 2> $out/cfg_${tag}_layers.err || fail $out/cfg_${tag}_layers.err
    python scripts/layer_roofline.py $out/cfg_${tag}_layers.txt --batch $b $args > $out/cfg_${tag}_roofline.txt
  done
}
t_runpy() {
  # the reference CLI at the headline shape over the native raw-frame reader (--num_workers 0 selects it): bench.py's
  # host corpus (96 decoded clips) linked 20x into a 1920-video split; --synthetic would measure CPU clip generation
  timeout -k 10 400 python bench.py --source host --steps 2 --warmup 1 > $out/runpy_corpus.json 2> $out/runpy_corpus.err || fail $out/runpy_corpus.err
  local src=/tmp/pva_bench_corpus/64x256x340_96/train dst=/tmp/pva_runpy_corpus c f b r
  rm -rf $dst && mkdir -p $dst/train
  for c in $(ls $src); do
    mkdir -p $dst/train/$c
    for f in $src/$c/*.npy; do b=$(basename $f .npy); for r in $(seq 0 19); do ln -s $f $dst/train/$c/${b}_$r.npy; done; done
  done
  ln -s $dst/train $dst/val
  timeout -k 10 600 python -u run.py --data_dir $dst --is_slowfast --num_frames 32 --sampling_rate 2 --crop_size 224 \
    --batch_size $B --gradient_accumulation_steps 1 --mixed_precision ${PRECISION:-bf16} --num_epochs 3 \
    --limit_train_batches 10 --limit_val_batches 0 --num_workers 0 --output_dir /tmp/pva_run --quiet \
    > $out/run_py_${PRECISION:-bf16}.log 2>&1 || fail $out/run_py_${PRECISION:-bf16}.log
  grep -i "clips/s" $out/run_py_${PRECISION:-bf16}.log | tail -4
}

t_benches() {
  # bench.py once per ";"-separated argument set in $BENCHES (non-headline models / precisions)
  local i=0
  IFS=';' read -ra arms <<< "$BENCHES"
  for arm in "${arms[@]}"; do
    i=$((i+1))
    local envs=(PVA_TUNE_LOG=1) args=() tok
    for tok in $arm; do if [[ $tok == PVA_*=* ]]; then envs+=("$tok"); else args+=("$tok"); fi; done
    env "${envs[@]}" timeout -k 10 500 python bench.py "${args[@]}" > $out/benches$i.json 2> $out/benches$i.err || fail $out/benches$i.err
    echo "$arm: $(cat $out/benches$i.json)"
  done
}
t_kstats() {
  # rocprofv3 per-kernel statistics of bench.py $KSTATS_ARGS (3 timed steps): top kernels by total time
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kstats -o k -- python3 bench.py --steps 3 --warmup 1 $KSTATS_ARGS > $out/kstats.log 2>&1 || fail $out/kstats.log
  local f
  f=$(ls $out/kstats/*/k_kernel_stats.csv $out/kstats/k_kernel_stats.csv 2>/dev/null | head -1)
  cp "$f" $out/kernel_stats.csv
  rm -rf $out/kstats
  python3 - "$out/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} launches")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d}  {r['Name'][:110]}")
PY
}
t_losstraj() {
  # bench recipe through the fused bf16 and the native fp32 executors side by side (scripts/diag_loss_trajectory.py)
  timeout -k 10 600 python -u scripts/diag_loss_trajectory.py ${LT_ARGS:---batch 48 --steps 8} > $out/loss_trajectory.jsonl 2> $out/loss_trajectory.err || fail $out/loss_trajectory.err
  tail -1 $out/loss_trajectory.jsonl
}
t_stock() {
  # stock PyTorch-ROCm eager baselines (scripts/baseline_torch.py), one run per ";"-separated argument set
  local i=0
  IFS=';' read -ra arms <<< "${STOCK:---dtype bf16 --batch 32}"
  for arm in "${arms[@]}"; do
    i=$((i+1))
    timeout -k 10 300 python -u scripts/baseline_torch.py --steps ${STEPS:-8} --warmup 3 $arm >> $out/stock.jsonl 2> $out/stock$i.err || fail $out/stock$i.err
  done
  cat $out/stock.jsonl
}
t_lab() {
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=fast -I csrc/kernels tools/gemm_lab.hip -o /tmp/gemm_lab > $out/lab_build.log 2>&1 || fail $out/lab_build.log
  local sh shapes
  shapes="${LAB_SHAPES:-250880,1024,1024 62720,512,3072 250880,256,768}"
  for sh in $shapes; do
    IFS=',' read -r m n k <<< "$sh"
    echo "shape $m $n $k" >> $out/lab.txt
    timeout -k 10 120 /tmp/gemm_lab $m $n $k 20 0 >> $out/lab.txt 2>&1 || fail $out/lab.txt
    timeout -k 10 120 /tmp/gemm_lab $m $n $k 20 1 >> $out/lab.txt 2>&1 || fail $out/lab.txt
  done
  cat $out/lab.txt
  if [ -n "$LAB_PMC" ]; then
    for sh in $shapes; do
      IFS=',' read -r m n k <<< "$sh"
      for hot in 0 1; do
        timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out/labpmc/${m}_${hot} -o p -- /tmp/gemm_lab $m $n $k 5 $hot $LAB_PMC > $out/labpmc_${m}_${hot}.log 2>&1 || fail $out/labpmc_${m}_${hot}.log
        timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $out/labpmc2/${m}_${hot} -o p -- /tmp/gemm_lab $m $n $k 5 $hot $LAB_PMC > $out/labpmc2_${m}_${hot}.log 2>&1 || fail $out/labpmc2_${m}_${hot}.log
      done
    done
  fi
}

for task in "$@"; do
  echo "== $task"
  "t_$task"
done
