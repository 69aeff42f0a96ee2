export OUT=r6_dpp4
bash scripts/gpu_run.sh smoke tests bench
