# Round pass on the GPU box: GPU tests, smoke, then the default bench line.
# usage: bash tools/gpu_pass.sh TAG [pytest -k expr]
set -e
O=gpurun_out/$1
mkdir -p $O
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err
