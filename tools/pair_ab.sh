# Same-box A/B of env variants on the full forward (kbench) with per-kernel times.
# usage (on the box): bash tools/pair_ab.sh "QCN_FC_HEAD=fused" "QCN_FC_HEAD=linear" ...
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pab
cd /tmp && export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/pab/$i -o run -- python3 $R/tools/kbench.py ${KB:-1024} 100 > $R/gpurun_out/pab/$i.log 2>&1
  echo "== $E"; grep "M img/s" $R/gpurun_out/pab/$i.log | tail -1
  python3 - "$R/gpurun_out/pab/$i/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "copyBuffer" in r["Name"]:
        continue
    print("  %-60s %6s %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1000))
PY
  rm -f $R/gpurun_out/pab/$i/run_kernel_trace.csv
done
