# Same-box A/B of one compile-time flag through conv_stamp.hip (same source).
# usage (on the box, from the repo root): bash tools/micro/flag_ab.sh "-DFLAG" [reps]
set -e
FL=$1; N=${2:-2}
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS -Iinclude -Iconvnet-quantization_amd/csrc"
hipcc $F tools/micro/conv_stamp.hip -o /tmp/stamp_a
hipcc $F $FL tools/micro/conv_stamp.hip -o /tmp/stamp_b
for i in $(seq $N); do
  echo "=== base"; timeout -k 10 60 /tmp/stamp_a | grep "us/launch"
  echo "=== $FL";  timeout -k 10 60 /tmp/stamp_b | grep "us/launch"
done
