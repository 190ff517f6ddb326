# the four-wave LSTM forward over ablation builds (tools/ablib)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
for v in a NOHS NOACTS; do
  SGG_LIB=$R/tools/ablib/libsgg_$v.so timeout -k 10 120 python tools/bench_kernels.py mwf 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || { echo FAIL; exit 1; }
done
