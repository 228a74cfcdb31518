# r03: one-launch classifier head (QCN_FC_FUSED=1, default) vs split-K +
# finisher launches: head / headline / QDQ GPU tests at both, kbench A/B at
# batch 1024 and 256, and the two bench workloads.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_fc
mkdir -p $O
for F in 1 0; do
  QCN_FC_FUSED=$F timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_models.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t$F.log 2>&1 || { tail -30 $O/t$F.log; exit 1; }
  echo "QCN_FC_FUSED=$F $(tail -1 $O/t$F.log)"
done
bash tools/pair_ab.sh QCN_FC_FUSED=1 QCN_FC_FUSED=0 QCN_FC_FUSED=1 QCN_FC_FUSED=0
KB=256 bash tools/pair_ab.sh QCN_FC_FUSED=1 QCN_FC_FUSED=0
for F in 1 0 1 0; do
  QCN_FC_FUSED=$F timeout -k 10 300 python bench.py --no-cpu --no-pmc --steps 50 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('convnet QCN_FC_FUSED=$F %.0f img/s %.4f ms' % (d['value'], d['ms_per_step']))"
  QCN_FC_FUSED=$F timeout -k 10 300 python bench.py --workload qdq --no-cpu --no-pmc --steps 50 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('qdq QCN_FC_FUSED=$F %.0f img/s %.4f ms' % (d['value'], d['ms_per_step']))"
done
