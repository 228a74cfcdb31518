# r03: ResNet GPU tests with 128-pixel tiles for thin convs, then same-box A/B
# of QCN_GEMM_THIN_K (0 = all convs on 256-pixel tiles) on the config-5 bench
# and per-layer times.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_thin
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for K in 0 256 512 0 256 512; do
  QCN_GEMM_THIN_K=$K timeout -k 10 300 python bench.py --workload resnet50 --steps 10 --warmup 3 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('thin_k=$K %8.0f img/s  conv %.3f ms  frac %.3f' % (d['value'], d['launch_ms']['conv'], d['roofline']['frac']))"
done
for K in 0 512; do
  QCN_GEMM_THIN_K=$K timeout -k 10 300 python tools/resnet_layers.py > $O/layers_$K.txt 2>&1
done
tail -n 2 $O/layers_0.txt $O/layers_512.txt
