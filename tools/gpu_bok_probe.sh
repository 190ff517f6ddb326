set -o pipefail
export TMPDIR=/tmp LSTM_PROBE_BOK=1
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bok_a -o run -- python3 $R/tools/lstm_probe.py 50 > $R/gpurun_out/bok_a.log 2>&1 &&
SGG_LSTM_NO_MFMA=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bok_b -o run -- python3 $R/tools/lstm_probe.py 50 > $R/gpurun_out/bok_b.log 2>&1
