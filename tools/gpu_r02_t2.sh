set -e
O=gpurun_out/r02_t2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -s -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err
