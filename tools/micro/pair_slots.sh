set -e
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -DQCN_STAMPS -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/pair_slots.hip -o /tmp/pair_slots
for S in 0; do
  for C in 64 128; do
    echo "=== cin=$C"
    timeout -k 10 60 /tmp/pair_slots $C
  done
done
