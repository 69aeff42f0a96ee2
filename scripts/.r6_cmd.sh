export OUT=r6_dpp
bash scripts/gpu_run.sh smoke tests bench
