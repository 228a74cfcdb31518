# Diagnostics: launch gaps of the forward loop and the configs[1] (QDQ,
# batch 256) bench line.  (The phase-stamp harness used in round 1 and early
# round 2 was removed together with its hooks in the product kernels; its data
# stays under profiles/r02_diag_stamps.txt and profiles/r01_diag_*.)
# usage (on the box, from the repo root): bash tools/gpu_diag.sh TAG
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-diag}
mkdir -p $O
bash tools/gpu_trace_gaps.sh ${1:-diag}
timeout -k 10 300 python bench.py --workload qdq --no-pmc > $O/bench_qdq.json 2> $O/bench_qdq.err
