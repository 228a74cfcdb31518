# conv12 barrier-wait stamps at batch 1024 and 8192, then the v14 perf pass
set -e
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/cs
QCN_SWEEP12=1 timeout -k 10 60 /tmp/cs > gpurun_out/sweep_wait.txt 2>&1
timeout -k 10 900 bash tools/gpu_perf.sh v14
