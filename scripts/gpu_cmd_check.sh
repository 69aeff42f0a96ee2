set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 || { tail -40 gpurun_out/gt.log; exit 1; }
tail -3 gpurun_out/gt.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_cur.json 2> gpurun_out/bench_cur.err || { tail -30 gpurun_out/bench_cur.err; exit 1; }
cat gpurun_out/bench_cur.json
