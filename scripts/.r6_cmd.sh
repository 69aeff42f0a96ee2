export OUT=r6_full
bash scripts/gpu_run.sh smoke tests
