# A/B of two GAT encoder probe builds on one box (old, new, old, new)
set -o pipefail
cd $GRAFT_REPO_ROOT
for b in gatenc_probe_old gatenc_probe gatenc_probe_old gatenc_probe; do
  echo "== $b"; timeout -k 10 60 tools/bin/$b 64 20 1 | grep -E "us/launch|staged|mark  1 " || { echo PROBE_FAIL; exit 1; }
done
