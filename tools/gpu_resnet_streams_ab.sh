# ResNet-50 (config 5) bench with 1..4 HIP streams over the batch, same box.
# usage (on the box): bash tools/gpu_resnet_streams_ab.sh TAG
set -e
O=gpurun_out/${1:-rs}
mkdir -p $O
for s in 2 3 4 2 3; do
  timeout -k 10 300 python bench.py --workload resnet50 --no-cpu --no-pmc --streams $s > $O/s$s.json 2> $O/s$s.err
  python3 -c "
import json
d=json.loads([l for l in open('$O/s$s.json') if l.startswith('{')][0])
print('streams $s', round(d['value']), round(d['ms_per_step'], 3))" >> $O/ab.txt
done
