set -o pipefail
timeout -k 10 400 python bench.py --depth 101 --crop 256 --batch 32 --steps 5 --warmup 2 > gpurun_out/bench_r101.json 2> gpurun_out/bench_r101.err || { tail -20 gpurun_out/bench_r101.err; exit 1; }
timeout -k 10 400 python bench.py --frames 64 --batch 32 --steps 5 --warmup 2 > gpurun_out/bench_t64.json 2> gpurun_out/bench_t64.err || { tail -20 gpurun_out/bench_t64.err; exit 1; }
timeout -k 10 400 python scripts/baseline_torch.py --batch 8 --steps 5 --warmup 2 --depth 101 --crop 256 > gpurun_out/base_r101.json 2> gpurun_out/base_r101.err || true
cat gpurun_out/bench_r101.json gpurun_out/bench_t64.json gpurun_out/base_r101.json
