# Sweep one env knob over values on the same box, interleaved (boxes differ by
# up to ~12 %): bash tools/sweep_env.sh NAME "v1 v2 ..." REPS
set -e
NAME=$1; VALS=$2; N=${3:-2}
for i in $(seq $N); do
  for v in $VALS; do
    env $NAME=$v timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('%-24s %9.0f img/s  ' % ('$NAME=$v', d['value']) + ' '.join('%s=%.1f' % (n, v['ms']*1e3) for n, v in k.items()), flush=True)"
  done
done
