export OUT=r6_cfg2
bash scripts/gpu_run.sh cfg
