set -e
O=$GRAFT_REPO_ROOT/gpurun_out/stamps; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/conv_stamp_x
timeout -k 10 60 /tmp/conv_stamp_x > $O/base.txt 2>&1
for V in "-DQCN_EXP_NOCONS" "-DQCN_EXP_NOPROD"; do
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS $V -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/conv_stamp_y
timeout -k 10 60 /tmp/conv_stamp_y > $O/v$V.txt 2>&1
done
