# GPU tests matching a -k expression (arg 1), one pytest process
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-tk}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$1" > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" $O/tests.log | tail -25
exit $rc
