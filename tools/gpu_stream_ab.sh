# r03: ResNet GPU tests at the streaming kernel's defaults (K <= 512, K >= 128
# through the LDS ring) and with K = 128 in registers, then the config-5 bench.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_stream3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
QCN_STREAM_BL128=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread -k stream > $O/tbl.log 2>&1 || { tail -30 $O/tbl.log; exit 1; }
tail -1 $O/tbl.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('default: %8.0f img/s  %.3f ms/step' % (d['value'], d['ms_per_step']))"
done
