# In-situ price of grid-wide barriers at the end of the one launch (the
# classifier head's seams if it moved into the persistent launch): the product
# library against the probe variants built by
#   bash tools/build_variant.sh gp1 "-DQCN_GRID_PROBE=1 -DQCN_GRID_PROBE_N=1" tools/patches/grid_probe.patch  (flat counter, 1 barrier)
#   bash tools/build_variant.sh gp2 "-DQCN_GRID_PROBE=1 -DQCN_GRID_PROBE_N=2" tools/patches/grid_probe.patch  (flat, 2)
#   bash tools/build_variant.sh gt1 "-DQCN_GRID_PROBE=2 -DQCN_GRID_PROBE_N=1" tools/patches/grid_probe.patch  (two-level tree, 1)
#   bash tools/build_variant.sh gt2 "-DQCN_GRID_PROBE=2 -DQCN_GRID_PROBE_N=2" tools/patches/grid_probe.patch  (tree, 2)
# two interleaved rounds, one process per library.  usage (on the box): bash tools/gpu_grid_probe.sh TAG
set -e
O=gpurun_out/$1
mkdir -p $O
L=convnet-quantization_amd/qconvnet
QCN_LIB=$L/libqconvnet.so timeout -k 10 120 python tools/grid_probe_ab.py prod --save $O/logits.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
for r in 1 2; do
  for v in prod gp1 gt1 gp2 gt2; do
    if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
    QCN_LIB=$lib timeout -k 10 120 python tools/grid_probe_ab.py $v --check $O/logits.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
  done
done
cat $O/ab.txt
