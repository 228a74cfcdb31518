# Parity gate (conv / headline tests) then a same-box A/B of the working tree's
# library against tools/ab/libqconvnet_base.so (built from HEAD).
# usage: bash tools/gpu_ab.sh TAG [REPS]
set -e
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/parity.log 2>&1
bash tools/ab.sh "QCN_LIB=tools/ab/libqconvnet_base.so" "QCN_LIB=convnet-quantization_amd/qconvnet/libqconvnet.so" ${2:-3} > $O/ab.txt 2>&1
