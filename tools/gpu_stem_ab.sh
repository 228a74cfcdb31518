# r03: fused stem with 1 / 2 / 4 pool rows per band (QCN_STEM_P): stem tests
# at each, then the config-5 bench and the stem's single-stream time.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_stem
mkdir -p $O
for P in 1 2 4; do
  QCN_STEM_P=$P timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread -k "stem or bit_exact" > $O/t$P.log 2>&1 || { tail -30 $O/t$P.log; exit 1; }
  echo "P=$P $(tail -1 $O/t$P.log)"
done
for P in 2 1 4 2 1 4; do
  QCN_STEM_P=$P timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('QCN_STEM_P=$P: %8.0f img/s  %.3f ms/step' % (d['value'], d['ms_per_step']))"
done
for P in 1 2 4; do
  QCN_STEM_P=$P timeout -k 10 300 python tools/resnet_layers.py 2>/dev/null | grep "7x1" | sed "s/^/P=$P /"
done
