# Quick iteration on the GPU box: selected GPU tests, then a rocprofv3
# kernel-trace summary of tools/kbench.py.  usage: bash tools/gpu_iter.sh TAG "pytest -k expr" [B] [ITERS]
set -e
O=gpurun_out/$1
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$2" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py ${3:-1024} ${4:-200} > $GRAFT_REPO_ROOT/$O/kbench.log 2>&1
cd $GRAFT_REPO_ROOT && python3 tools/stats_summary.py $O/prof > $O/stats.txt 2>&1 || true
