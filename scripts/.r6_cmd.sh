export OUT=r6_magic
bash scripts/gpu_run.sh smoke tests bench
