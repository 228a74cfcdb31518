# Kernel traces of the default bench with the split-K head and the one-launch
# head (QCN_FC_HEAD=one): per-launch durations and gaps in timed region A.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_headtr}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for H in fused one; do
  QCN_FC_HEAD=$H timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/tr_$H -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pmc --steps 100 --warmup 20 > $O/bench_$H.json 2> $O/bench_$H.err
done
cd $GRAFT_REPO_ROOT
for H in fused one; do
  python3 tools/trace_gaps.py $O/tr_$H/run_kernel_trace.csv 20 100 > $O/gaps_$H.txt 2>&1 || true
  rm -f $O/tr_$H/run_kernel_trace.csv
done
