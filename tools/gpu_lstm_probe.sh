# phase probe of the four-wave encoder forward (tools/lstm_mw_probe.hip builds in tools/run/)
set -o pipefail
for v in "$@"; do
  for args in "2560 12 1 1" "1280 12 1 1"; do
    echo "== $v $args"; timeout -k 10 60 tools/run/lstm_probe_$v $args || { echo PROBE_FAIL; exit 1; }
  done
done
