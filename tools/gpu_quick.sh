# Quick GPU loop: parity gate then bench (no CPU baseline) and a kernel trace.
# usage (on the box, from the repo root): bash tools/gpu_quick.sh TAG
set -e
TAG=${1:-quick}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/trace.log 2>&1
echo done > $O/DONE
