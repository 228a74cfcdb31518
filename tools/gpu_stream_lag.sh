# ResNet-50 (batch 512, two streams) with slice 1 started N launches behind
# slice 0 (bench --stream-lag N), N = 0 (the product) .. 3, two rounds, same
# box, after the run_streams tests.  usage (on the box): bash tools/gpu_stream_lag.sh TAG
set -e
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -x -q -k run_streams --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for r in 1 2; do
  for lag in 0 1 2 3; do
    timeout -k 10 300 python bench.py --workload resnet50 --no-cpu --no-pmc --stream-lag $lag > $O/lag$lag.$r.json 2> $O/lag$lag.$r.err
    python -c "import json; d=json.loads(open('$O/lag$lag.$r.json').read().strip().splitlines()[-1]); print('lag $lag round $r', round(d['value']), d['ms_per_step'])" | tee -a $O/ab.txt
  done
done
