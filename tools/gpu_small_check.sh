# Small-batch conv5+6 (one image per 8-wave workgroup) and one-launch convs
# check on the box: the pair / config-2 / headline GPU tests, then the
# host-cost probe (device time per forward, static / QDQ) for the product
# library and for the r03 cout-split conv5+6 variant (libqconvnet_sm0.so, if
# built), and the one-launch vs three-launch A/B at batch 1024.
# usage (on the box): bash tools/gpu_small_check.sh TAG
set -e
O=gpurun_out/${1:-small}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "one_launch or headline or pair or config2" --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python tools/host_cost.py > $O/host_cost.txt 2>&1
timeout -k 10 300 python tools/host_cost.py --three > $O/host_cost_three.txt 2>&1
if [ -f convnet-quantization_amd/qconvnet/libqconvnet_sm0.so ]; then
  QCN_LIB=convnet-quantization_amd/qconvnet/libqconvnet_sm0.so timeout -k 10 300 python tools/host_cost.py --three > $O/host_cost_sm0_three.txt 2>&1
fi
timeout -k 10 300 python tools/c16_ab.py > $O/c16_ab.txt 2>&1
timeout -k 10 300 python tools/clock_probe.py --batch 1024 > $O/clock_1024.txt 2>&1
timeout -k 10 300 python tools/clock_probe.py --batch 256 --workload qdq > $O/clock_qdq256.txt 2>&1
