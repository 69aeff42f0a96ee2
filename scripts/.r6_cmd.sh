export OUT=r6_aff
mkdir -p gpurun_out/r6_aff && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6_aff/kern.log 2>&1 && tail -1 gpurun_out/r6_aff/kern.log && bash scripts/gpu_run.sh bench layers
