# Kernel trace of the default bench (trained-model weights) with per-dispatch
# start / end kept: per-launch durations and gaps inside timed region A.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_bgaps}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pmc > $O/bench.json 2> $O/bench.err
cd $GRAFT_REPO_ROOT
python3 tools/trace_gaps.py $O/trace/run_kernel_trace.csv 10 50 > $O/gaps_regionA.txt
python3 tools/trace_gaps.py $O/trace/run_kernel_trace.csv 60 50 > $O/gaps_regionB.txt
rm -f $O/trace/run_kernel_trace.csv
