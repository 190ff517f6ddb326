# LSTM four-wave forward: the Wu prefetch spread over the steps (new) vs all
# in the prologue (old), A/B on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
for a in "old 2560 12 1" "u1 2560 12 1" "old 1280 12 1" "u1 1280 12 1" "old 2560 12 1" "u1 2560 12 1" "u1 2560 4 1"; do
  set -- $a
  echo "== $a"; timeout -k 10 60 tools/bin/lstm_mw_probe_$1 $2 $3 $4 | head -4 || { echo PROBE_FAIL; exit 1; }
done
