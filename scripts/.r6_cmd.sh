export OUT=r6_end2
bash scripts/gpu_run.sh smoke tests bench
