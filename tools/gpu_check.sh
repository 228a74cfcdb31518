# GPU tests (all), then the default bench line.  usage: bash tools/gpu_check.sh TAG
set -e
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err
