export OUT=r6_wgp
bash scripts/gpu_run.sh smoke tests bench
