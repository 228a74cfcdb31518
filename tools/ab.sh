# A/B two configurations on the same box (boxes differ by up to ~12 %).  Each
# argument is a string of env assignments, e.g.
#   bash tools/ab.sh "QCN_LIB=tools/ab/libqconvnet_a.so" "" 3 ["--workload qdq"]
set -e
A=$1; B=$2; N=${3:-3}; X=${4:-}
for i in $(seq $N); do
  for E in "$A" "$B"; do
    env $E timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu --no-pmc --no-extra $X 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('%-36s %9.0f img/s  ' % ('[$E]'[-36:], d['value']) + ' '.join('%s=%.1f' % (n, v['ms']*1e3) for n, v in k.items()))"
  done
done
