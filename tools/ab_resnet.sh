# Same-box A/B of the ResNet-50 workload (configs[4]) between two libraries.
# usage: bash tools/ab_resnet.sh LIB_A LIB_B [REPS]
set -e
A=$1; B=$2; N=${3:-2}
for i in $(seq $N); do
  for L in "$A" "$B"; do
    QCN_LIB=$L timeout -k 10 300 python bench.py --workload resnet50 --steps 10 --warmup 3 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('%-40s %8.0f img/s  conv %.3f ms  frac %.3f' % ('$L'[-40:], d['value'], d['launch_ms']['conv'], d['roofline']['frac']))"
  done
done
