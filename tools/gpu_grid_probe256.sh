# The grid-barrier probe (tools/gpu_grid_probe.sh) at configs[1]'s batch 256,
# where the one launch is convnet_convs_sm_kernel (one image per workgroup):
# the per-layer QDQ net and the static net, product vs the tree-barrier
# variants gt1 / gt2.  usage (on the box): bash tools/gpu_grid_probe256.sh TAG
set -e
O=gpurun_out/$1
mkdir -p $O
L=convnet-quantization_amd/qconvnet
for m in --qdq ""; do
  QCN_LIB=$L/libqconvnet.so timeout -k 10 120 python tools/grid_probe_ab.py prod 256 2000 3 $m --save $O/logits$m.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
  for r in 1 2; do
    for v in prod gt1 gt2; do
      if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
      QCN_LIB=$lib timeout -k 10 120 python tools/grid_probe_ab.py $v$m 256 2000 3 $m --check $O/logits$m.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
    done
  done
done
cat $O/ab.txt
