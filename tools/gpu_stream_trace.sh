# r03: kernel-trace stats of the config-5 bench (back-to-back forwards, no
# per-launch events) with the streaming 1x1 kernel off / K<=128 / K<=256.
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r03_strace
mkdir -p $O
for S in 0 128 256 0 128 256; do
  QCN_GEMM_STREAM=$S timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('stream=$S %8.0f img/s  %.3f ms/step' % (d['value'], d['ms_per_step']))"
done
cd /tmp && export TMPDIR=/tmp
for S in 0 128 256; do
  QCN_GEMM_STREAM=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/k$S -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc > $O/k$S.log 2>&1
done
cd $GRAFT_REPO_ROOT
for S in 0 128 256; do
  echo "== QCN_GEMM_STREAM=$S"
  python3 - $O/k$S <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f"  {r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.1f} us  {float(r['TotalDurationNs'])/tot*100:5.1f} %")
print(f"  total {tot/1e6:.1f} ms")
PY
done
