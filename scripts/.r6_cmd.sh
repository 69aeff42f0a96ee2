timeout -k 10 400 python -u scripts/dp_det_check.py --reps 3 --load --single-load
