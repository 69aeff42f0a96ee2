export OUT=r6_wnarrow
mkdir -p gpurun_out/r6_wnarrow && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad or narrow or gram or fold" > gpurun_out/r6_wnarrow/kern.log 2>&1 && tail -1 gpurun_out/r6_wnarrow/kern.log && bash scripts/gpu_run.sh bench
