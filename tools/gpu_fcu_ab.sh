# Same-box A/B of the split-K load batch (QCN_FC_U) on the default bench:
# (r06: the QCN_JOIN_AFF / QCN_FC_U switches this used were removed from csrc/; to rerun, add them back as a patch under tools/patches/.)
# product (U = 4) vs libqconvnet_fcu8.so / _fcu2.so, two rounds.
# usage (on the box): bash tools/gpu_fcu_ab.sh TAG
set -e
O=gpurun_out/${1:-fcu}
mkdir -p $O
L=convnet-quantization_amd/qconvnet
for r in 1 2; do
  for v in prod fcu8 fcu2; do
    if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
    QCN_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-pmc --steps 400 > $O/$v.$r.json 2> $O/$v.$r.err
    python3 -c "
import json,sys
d=json.loads([l for l in open('$O/$v.$r.json') if l.startswith('{')][0])
print('$v', round(d['value']), ' '.join('%s=%.2f' % (k, v['ms']*1e3) for k, v in d['kernels'].items()))" >> $O/ab.txt
  done
done
