# r03: parity (pair / headline / conv56 / qdq tests) with the small-batch pair
# forms, then same-box A/B at batch 256 (kbench under rocprof) and config 2.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pair or headline or conv56 or qdq" > gpurun_out/r03_small_t.log 2>&1 || { tail -40 gpurun_out/r03_small_t.log; exit 1; }
tail -2 gpurun_out/r03_small_t.log
KB=256 bash tools/pair_ab.sh "QCN_SMALL34=0" "QCN_SMALL34=1" "QCN_SMALL34=0" "QCN_SMALL34=1"
for E in "QCN_SMALL34=0" "QCN_SMALL34=1" "QCN_SMALL34=0" "QCN_SMALL34=1"; do
  env $E timeout -k 10 300 python bench.py --workload qdq --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('qdq [$E] %.0f img/s ' % d['value'] + ' '.join('%s=%.1f' % (n, v['ms']*1e3) for n, v in k.items()))"
done
for W in qdq convnet; do
  timeout -k 10 300 python bench.py --workload $W --no-cpu --no-pmc --pipeline 2 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$W one stream %.0f img/s; 2 batches in flight %.0f img/s (%.4f ms/batch)' % (d['value'], d['pipelined']['value'], d['pipelined']['ms_per_batch']))"
done
