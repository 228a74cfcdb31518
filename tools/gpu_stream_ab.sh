# r03: K = 64 1x1 convs through the LDS ring (QCN_STREAM_BL64) — ResNet tests
# with it, same-box config-5 bench A/B, then the bench's stream count 1/2/3.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_stream5
mkdir -p $O
QCN_STREAM_BL64=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for V in 0 1 0 1; do
  QCN_STREAM_BL64=$V timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('QCN_STREAM_BL64=$V: %8.0f img/s  %.3f ms/step' % (d['value'], d['ms_per_step']))"
done
for S in 1 2 3 1 2 3; do
  timeout -k 10 300 python bench.py --workload resnet50 --streams $S --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('streams=$S: %8.0f img/s  %.3f ms/step' % (d['value'], d['ms_per_step']))"
done
for V in 0 1; do
  QCN_STREAM_BL64=$V timeout -k 10 300 python tools/resnet_layers.py > $O/layers_$V.txt 2>&1
done
paste $O/layers_0.txt $O/layers_1.txt | grep -v amdgpu.ids | awk -F'\t' '{printf "%-92s | %s\n", $1, substr($2,39,8)}' | grep "56    64"
