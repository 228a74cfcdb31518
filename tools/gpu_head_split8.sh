# The classifier head with an 8-way K split below 1024 rows: the headline /
# parity GPU tests, then product vs the previous library (libqconvnet_pre.so,
# 4-way split), configs[1] (QDQ, batch 256) and the static net at 256 and
# 1024, two interleaved rounds on tools/grid_probe_ab.py.
# usage (on the box): bash tools/gpu_head_split8.sh TAG
set -e
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
L=convnet-quantization_amd/qconvnet
for cfg in "256 2000 3 --qdq" "256 2000 3" "1024 1000 3"; do
  QCN_LIB=$L/libqconvnet_pre.so timeout -k 10 120 python tools/grid_probe_ab.py pre $cfg --save $O/logits.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
  for r in 1 2; do
    for v in pre prod; do
      if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
      QCN_LIB=$lib timeout -k 10 120 python tools/grid_probe_ab.py $v $cfg --check $O/logits.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
    done
  done
done
cat $O/ab.txt
