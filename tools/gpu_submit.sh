#!/bin/bash
# usage (from the repo root): bash tools/gpu_submit.sh OUTFILE <gpurun args...>
# submit a gpurun call; re-submit only when the pool had no slot/box (nothing ran, nothing charged)
out=$1; shift
for a in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "nothing was charged\|has no free box right now" $out && ! grep -q "status=ok\|status=fail" $out; then
    sleep 150
    continue
  fi
  exit $rc
done
exit $rc
