# r03: software-pipelined stream steps (QCN_STREAM_PIPE=1): strip t+1 MFMAs
# interleaved with strip t requant. ResNet tests with it on, same-box config-5
# bench A/B and per-layer times.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_stream_pipe
mkdir -p $O
QCN_STREAM_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for V in 0 1 0 1; do
  QCN_STREAM_PIPE=$V timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('QCN_STREAM_PIPE=$V: %8.0f img/s  %.3f ms/step' % (d['value'], d['ms_per_step']))"
done
for V in 0 1; do
  QCN_STREAM_PIPE=$V timeout -k 10 300 python tools/resnet_layers.py > $O/layers_$V.txt 2>&1
done
paste $O/layers_0.txt $O/layers_1.txt | grep -v amdgpu.ids | awk -F'\t' '{printf "%-92s | %s\n", $1, substr($2,39,8)}' | grep -E "1x1|total"
