# The one launch with ScratchSize 0 (tid laundered in the setup code): the
# headline / pair / W4 GPU tests, then product vs the previous library
# (libqconvnet_pre.so), three interleaved rounds on tools/grid_probe_ab.py.
# usage (on the box): bash tools/gpu_scratch0_check.sh TAG
set -e
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_w4.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
L=convnet-quantization_amd/qconvnet
QCN_LIB=$L/libqconvnet_pre.so timeout -k 10 120 python tools/grid_probe_ab.py pre --save $O/logits.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
for r in 1 2 3; do
  for v in pre prod; do
    if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
    QCN_LIB=$lib timeout -k 10 120 python tools/grid_probe_ab.py $v --check $O/logits.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
  done
done
cat $O/ab.txt
