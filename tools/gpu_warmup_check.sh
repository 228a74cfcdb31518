# r03: bench.py with the time-based ramp warmup — the driver's own command
# (--steps 20 --warmup 5) next to a long steady-state run, all workloads,
# and bench.py's two-rank rehearsal test.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_warmup
mkdir -p $O
summ() { python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$1', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,1), 'us/step, warmup steps run', d.get('warmup_steps_run'))"; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | summ "convnet 20/5"
  timeout -k 10 300 python bench.py --gpus 1 --steps 1000 --warmup 100 --no-cpu --no-pmc 2>/dev/null | summ "convnet 1000/100"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --warmup-min-ms 0 --no-cpu --no-pmc 2>/dev/null | summ "convnet 20/5 no ramp"
done
timeout -k 10 300 python bench.py --workload qdq --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | summ "qdq 20/5"
timeout -k 10 300 python bench.py --workload qdq --steps 1000 --warmup 100 --no-cpu --no-pmc 2>/dev/null | summ "qdq 1000/100"
timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | summ "resnet 20/5"
timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --warmup-min-ms 0 --no-cpu --no-pmc 2>/dev/null | summ "resnet 20/5 no ramp"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
