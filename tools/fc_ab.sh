# fc head A/B: per-kernel times of the forward under rocprofv3 for env variants.
# usage (on the box): bash tools/fc_ab.sh "QCN_FC_U=4" "QCN_FC_U=8"
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/fcab/$i -o run -- python3 $R/tools/kbench.py 1024 100 > $R/gpurun_out/fcab/$i.log 2>&1
  echo "== $E"; grep "M img/s" $R/gpurun_out/fcab/$i.log | tail -1
  python3 - "$R/gpurun_out/fcab/$i/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("  %-60s %6s %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1000))
PY
  rm -f $R/gpurun_out/fcab/$i/run_kernel_trace.csv
done
