# Diagnostic variants of the pair kernels (outputs wrong by design): no weight
# DMA in the main loop / no A-epilogue requant.
set -e
for V in "" "-DQCN_EXP_NODMA" "-DQCN_EXP_NOEPIA" "-DQCN_EXP_NODMA -DQCN_EXP_NOEPIA"; do
  echo "=== variant: $V"
  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS $V -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/conv_stamp_x
  timeout -k 10 60 /tmp/conv_stamp_x | head -8
done
