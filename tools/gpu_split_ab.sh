# r03: parity (pair / headline / conv56 tests) with the cout-split conv5+6, then
# same-box A/B of the split threshold at batch 256 and 512, and config 2.
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pair or headline or conv56 or qdq" > gpurun_out/r03_split_t.log 2>&1 || { tail -40 gpurun_out/r03_split_t.log; exit 1; }
tail -2 gpurun_out/r03_split_t.log
KB=256 bash tools/pair_ab.sh "QCN_SPLIT56=0" "QCN_SPLIT56=2" "QCN_SPLIT56=0" "QCN_SPLIT56=2"
KB=512 bash tools/pair_ab.sh "QCN_SPLIT56=0" "QCN_SPLIT56=2"
for E in "QCN_SPLIT56=0" "QCN_SPLIT56=2"; do
  env $E timeout -k 10 300 python bench.py --workload qdq --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('qdq [$E] %.0f img/s ' % d['value'] + ' '.join('%s=%.1f' % (n, v['ms']*1e3) for n, v in k.items()))"
done
