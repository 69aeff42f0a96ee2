timeout -k 10 700 python -u scripts/.r6_detchk.py
