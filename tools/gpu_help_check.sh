# Fill-period helper (QCN_WS_HELP) check on the box: pair / one-launch /
# headline / config-2 GPU tests, then the one-launch forward A/B product vs
# the -DQCN_WS_HELP=0 variant (tools/c16_ab.py under each library, two rounds),
# and the phase stamps of the pairs inside the one launch.
# usage (on the box): bash tools/gpu_help_check.sh TAG
set -e
O=gpurun_out/${1:-help}
mkdir -p $O
L=convnet-quantization_amd/qconvnet
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "one_launch or headline or pair or config2" --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
for r in 1 2; do
  for v in prod nohelp; do
    if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
    echo "## $v round $r" >> $O/ab.txt
    QCN_LIB=$lib timeout -k 10 200 python tools/c16_ab.py 1024 1000 3 2>&1 | grep -v amdgpu >> $O/ab.txt
  done
done
QCN_LIB=tools/clock/libqconvnet_clock.so timeout -k 10 200 python tools/p34_stamps.py 1024 2 > $O/stamps.txt 2>&1
