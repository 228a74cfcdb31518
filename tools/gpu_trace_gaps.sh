# Kernel trace of the forward loop (tools/kbench.py) with per-dispatch start /
# end kept, then the per-launch durations and the gaps between launches.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_gaps}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py 1024 200 > $O/kbench.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/trace_gaps.py $O/trace/run_kernel_trace.csv > $O/gaps.txt
rm -f $O/trace/run_kernel_trace.csv
