# One-form residual join check on the box: the ResNet GPU tests, then the
# (r06: the QCN_JOIN_AFF / QCN_FC_U switches this used were removed from csrc/; to rerun, add them back as a patch under tools/patches/.)
# ResNet-50 bench (two streams, batch 512) product vs the -DQCN_JOIN_AFF=0
# variant, two rounds, and the per-layer times of both.
# usage (on the box): bash tools/gpu_join_check.sh TAG
set -e
O=gpurun_out/${1:-join}
mkdir -p $O
L=convnet-quantization_amd/qconvnet
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "resnet or stream or gemm" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for r in 1 2; do
  for v in prod jaff0; do
    if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
    QCN_LIB=$lib timeout -k 10 300 python bench.py --workload resnet50 --no-cpu --no-pmc > $O/$v.$r.json 2> $O/$v.$r.err
    python3 -c "
import json
d=json.loads([l for l in open('$O/$v.$r.json') if l.startswith('{')][0])
print('$v', round(d['value']), round(d['ms_per_step'], 3))" >> $O/ab.txt
  done
done
QCN_LIB=$L/libqconvnet.so timeout -k 10 300 python tools/resnet_layers.py > $O/layers_prod.txt 2>&1
QCN_LIB=$L/libqconvnet_jaff0.so timeout -k 10 300 python tools/resnet_layers.py > $O/layers_jaff0.txt 2>&1
