# host-side trace of graphed real-data training: one
# rocprofv3 --sys-trace run of tools/realdata_graph_probe.py (the program
# itself after --), per-iteration host windows -> tools/systrace_stall.py
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-rd_sys}
mkdir -p $O
cd /tmp
SGG_PROBE_MARKS=$O/marks.json timeout -k 10 300 rocprofv3 --sys-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/realdata_graph_probe.py 60 > $O/probe.txt 2> $O/trace.err || { echo TRACE_FAIL; tail -20 $O/trace.err; exit 1; }
cat $O/probe.txt
python3 $R/tools/systrace_stall.py $O/trace $O/marks.json 4 > $O/stall.txt 2>&1
cat $O/stall.txt
rm -rf $O/trace
