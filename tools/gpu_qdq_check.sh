# QDQ-path check on the box: the GPU tests that run QDQ hand-offs, then the
# config-2 bench line (no CPU baseline, no counters) and the host-cost probe.
# usage (on the box): bash tools/gpu_qdq_check.sh TAG
set -e
O=gpurun_out/${1:-qdq}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "qdq or QDQ or config2 or pair or conv12 or headline" --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --workload qdq --no-cpu --no-pmc > $O/bench_qdq.json 2> $O/bench_qdq.err
timeout -k 10 300 python tools/host_cost.py > $O/host_cost.txt 2>&1
