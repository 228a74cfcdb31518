# Diagnostics: conv/pair phase stamps (random data), launch gaps of the
# forward loop, and the configs[1] (QDQ, batch 256) bench line.
# usage (on the box, from the repo root): bash tools/gpu_diag.sh TAG
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-diag}
mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS -Iinclude \
  -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/stamp
timeout -k 10 120 /tmp/stamp > $O/stamps.txt 2>&1
bash tools/gpu_trace_gaps.sh ${1:-diag}
timeout -k 10 300 python bench.py --workload qdq --no-pmc > $O/bench_qdq.json 2> $O/bench_qdq.err
