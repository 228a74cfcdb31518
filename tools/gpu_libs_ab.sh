# Same-box A/B of diagnostic library variants (libqconvnet_VARIANT.so, "prod" =
# the product library) on tools/grid_probe_ab.py: back-to-back forward time and
# per-launch HIP-event means at batch 1024, logits checked bit for bit against
# the product's, two interleaved rounds, one process per library.
# usage (on the box): bash tools/gpu_libs_ab.sh TAG VARIANT...
set -e
O=gpurun_out/$1
shift
mkdir -p $O
L=convnet-quantization_amd/qconvnet
QCN_LIB=$L/libqconvnet.so timeout -k 10 120 python tools/grid_probe_ab.py prod --save $O/logits.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
for r in 1 2; do
  for v in "$@"; do
    if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
    QCN_LIB=$lib timeout -k 10 120 python tools/grid_probe_ab.py $v --check $O/logits.npy 2>&1 | grep -v amdgpu >> $O/ab.txt
  done
done
cat $O/ab.txt
