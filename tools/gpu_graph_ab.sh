# r03: QDQ / conv56 / headline parity, then bench.py with and without HIP-graph
# replay for config 2 (batch 256) and the headline (batch 1024), same box.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "qdq or conv56 or headline" > gpurun_out/r03_g_t.log 2>&1 || { tail -30 gpurun_out/r03_g_t.log; exit 1; }
tail -2 gpurun_out/r03_g_t.log
line() {
  python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('$1 %.0f img/s %.4f ms ' % (d['value'], d['ms_per_step']) + ' '.join('%s=%.1f' % (n, v['ms']*1e3) for n, v in k.items()))"
}
for A in --graph --no-graph --graph; do
  timeout -k 10 300 python bench.py --workload qdq --no-cpu --no-pmc $A 2>/dev/null | line "qdq $A"
done
for A in --graph --no-graph --graph --no-graph; do
  timeout -k 10 300 python bench.py --no-cpu --no-pmc $A 2>/dev/null | line "convnet $A"
done
