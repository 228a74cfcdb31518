# K = 1024 streaming 1x1 (conv1x1_k1024_kernel) on the box: the ResNet GPU
# tests, then ResNet-50 (batch 512, two streams) product vs the previous
# library (libqconvnet_rn0.so: conv_gemm_kernel for those convs), two rounds,
# then the per-layer times of the product.  usage: bash tools/gpu_k1024_check.sh TAG
set -e
O=gpurun_out/$1
mkdir -p $O
L=convnet-quantization_amd/qconvnet
timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
for r in 1 2; do
  for v in rn0 prod; do
    if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
    QCN_LIB=$lib timeout -k 10 300 python bench.py --workload resnet50 --no-cpu --no-pmc > $O/bench_$v$r.json 2> $O/bench_$v$r.err
    python -c "import json; d=json.loads(open('$O/bench_$v$r.json').read().strip().splitlines()[-1]); print('$v round $r', round(d['value']), d['ms_per_step'])" | tee -a $O/ab.txt
  done
done
QCN_LIB=$L/libqconvnet.so timeout -k 10 200 python tools/resnet_layers.py > $O/layers_prod.txt 2>&1
QCN_LIB=$L/libqconvnet_rn0.so timeout -k 10 200 python tools/resnet_layers.py > $O/layers_rn0.txt 2>&1
echo done
