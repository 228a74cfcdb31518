# r03: conv12's last tile on all eight waves (QCN_C12_SPLITLAST=1): headline /
# QDQ / model GPU tests with it on, then same-box A/B of bench.py (batch 1024
# and config 2) and rocprofv3 kernel stats of kbench at batch 1024 and 256.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_c12split
mkdir -p $O
QCN_C12_SPLITLAST=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_models.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
summ() { python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$1', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v['ms']*1e3,1) for k,v in d.get('kernels',{}).items()})"; }
for i in 1 2; do
  for V in 0 1; do
    QCN_C12_SPLITLAST=$V timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-pmc 2>/dev/null | summ "b1024 SPLITLAST=$V"
    QCN_C12_SPLITLAST=$V timeout -k 10 300 python bench.py --workload qdq --steps 200 --warmup 20 --no-cpu --no-pmc 2>/dev/null | summ "qdq b256 SPLITLAST=$V"
  done
done
cd /tmp && export TMPDIR=/tmp
for V in 0 1; do
  for B in 1024 256; do
    QCN_C12_SPLITLAST=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/p${V}_$B -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py $B 100 > $O/p${V}_$B.log 2>&1
    python3 -c "
import csv
for r in csv.DictReader(open('$O/p${V}_$B/run_kernel_stats.csv')):
    if 'conv12' in r['Name']: print('rocprof b$B SPLITLAST=$V', r['Name'][:40], round(float(r['AverageNs'])/1e3, 2), 'us')"
  done
done
find $O -name '*_kernel_trace.csv' -delete
