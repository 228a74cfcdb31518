# Kernel trace summary of the bench (usage: bash tools/gpu_trace.sh TAG [bench args])
set -e
TAG=${1:-trace}; shift || true
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu "$@" > $O/trace.log 2>&1
python3 - "$O/trace/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-70s %6s %9.2f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1000))
PY
