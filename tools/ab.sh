# A/B two builds of libqconvnet.so on the same box (boxes differ by up to ~12 %):
#   bash tools/ab.sh tools/ab/libqconvnet_a.so convnet-quantization_amd/qconvnet/libqconvnet.so [rounds]
set -e
A=$1; B=$2; N=${3:-3}
for i in $(seq $N); do
  for L in "$A" "$B"; do
    QCN_LIB=$L timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('%-48s %9.0f img/s  ' % ('$L'[-48:], d['value']) + ' '.join('%s=%.1f' % (n, v['ms']*1e3) for n, v in k.items()))"
  done
done
