# Small-batch conv5+6 (one image per 8-wave workgroup) check on the box: the
# pair / config-2 / headline GPU tests, then the host-cost probe (device time
# per forward at batch 128 / 256 static and QDQ, 1024).
# usage (on the box): bash tools/gpu_small_check.sh TAG
set -e
O=gpurun_out/${1:-small}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "one_launch or headline or pair or config2" --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python tools/host_cost.py > $O/host_cost.txt 2>&1
timeout -k 10 300 python tools/c16_ab.py > $O/c16_ab.txt 2>&1
