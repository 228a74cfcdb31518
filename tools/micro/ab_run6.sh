# per-XCD workgroup durations of every conv kernel (stamp harness), twice
set -e
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/cs
timeout -k 10 60 /tmp/cs > gpurun_out/xcd1.txt 2>&1
timeout -k 10 60 /tmp/cs > gpurun_out/xcd2.txt 2>&1
