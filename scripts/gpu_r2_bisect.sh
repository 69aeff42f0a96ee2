cd $GRAFT_REPO_ROOT
for k in f fres fw2 eb er d; do
  echo "== kinds=$k"
  PVA_PW_KINDS=$k timeout -k 10 120 python scripts/diag_ms_det.py 2>&1 | grep "ms=" | awk '{print $2, $3}' | tr '\n' ' '; echo
done
