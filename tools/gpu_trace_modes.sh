# Kernel trace of tools/kbench.py at batch B for the static and the QDQ
# model: per-launch durations and the gaps between launches of each.
# usage (on the box): bash tools/gpu_trace_modes.sh TAG [B]
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-modes}
B=${2:-256}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in static qdq; do
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/$m -o run -- python3 $R/tools/kbench.py $B 300 $m > $O/kbench_$m.log 2>&1
  python3 $R/tools/trace_gaps.py $O/$m/run_kernel_trace.csv > $O/gaps_$m.txt
  rm -f $O/$m/run_kernel_trace.csv
done
