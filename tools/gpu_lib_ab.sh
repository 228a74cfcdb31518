# Same-box A/B of diagnostic library variants on tools/host_cost.py (device
# time per forward, static / QDQ, batch 128 / 256 / 1024), two rounds.
# usage (on the box): bash tools/gpu_lib_ab.sh TAG VARIANT...   (libqconvnet_VARIANT.so; "prod" = product)
set -e
O=gpurun_out/$1
shift
mkdir -p $O
L=convnet-quantization_amd/qconvnet
for r in 1 2; do
  for v in "$@"; do
    if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
    echo "## $v round $r" >> $O/ab.txt
    QCN_LIB=$lib timeout -k 10 200 python tools/host_cost.py 2>&1 | grep -v amdgpu >> $O/ab.txt
  done
done
