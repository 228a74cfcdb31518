# Data dependence of the int8 conv kernels' speed (DVFS): same binary, activation fills.
set -e
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/conv_stamp_f
for F in rand zero mid relu; do
  echo "=== fill $F"
  QCN_FILL=$F timeout -k 10 60 /tmp/conv_stamp_f | grep -A1 "us/launch"
done
