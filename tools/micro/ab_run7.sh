# conv12 fused-vs-unfused parity over batch sizes
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k fused_conv12 > gpurun_out/par12.txt 2>&1
