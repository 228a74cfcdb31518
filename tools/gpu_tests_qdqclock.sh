# Full GPU test suite, then the config-2 (QDQ, batch 256) per-phase clock probe.
set -e
TAG=${1:-t}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python tools/clock_probe.py --workload qdq > $O/probe_qdq.json 2> $O/probe_qdq.txt
cat $O/probe_qdq.txt
