timeout -k 10 600 python -u scripts/dp_det_check.py --reps 5 --load
