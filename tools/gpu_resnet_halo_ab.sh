# r03: ResNet GPU tests with the patch-staged layer-1 3x3 convs, then per-layer
# times and the config-5 bench line with QCN_RESNET_HALO=0/1, same box.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_halo
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for H in 0 1; do
  QCN_RESNET_HALO=$H timeout -k 10 300 python tools/resnet_layers.py > $O/layers_$H.txt 2>&1
done
for H in 0 1 0 1; do
  QCN_RESNET_HALO=$H timeout -k 10 300 python bench.py --workload resnet50 --steps 10 --warmup 3 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('halo=$H %8.0f img/s  conv %.3f ms  frac %.3f' % (d['value'], d['launch_ms']['conv'], d['roofline']['frac']))"
done
grep "3x3    1   56" $O/layers_0.txt $O/layers_1.txt || true
tail -2 $O/layers_0.txt $O/layers_1.txt
