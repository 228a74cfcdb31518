# Same-box A/B over several library builds (tools/ab/libqconvnet_<tag>.so).
# usage: bash tools/ab_multi.sh REPS tag1 tag2 ...
set -e
N=$1; shift
for i in $(seq $N); do
  for T in "$@"; do
    QCN_LIB=tools/ab/libqconvnet_$T.so timeout -k 10 300 python bench.py ${BENCH_ARGS:-} --steps 100 --warmup 20 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('%-8s %9.0f img/s  ' % ('$T', d['value']) + ' '.join('%s=%.1f' % (n, v['ms']*1e3) for n, v in k.items()))"
  done
done
