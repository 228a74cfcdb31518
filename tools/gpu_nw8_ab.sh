# r03: 8-wave stream workgroups for wide 1x1 convs (QCN_STREAM_NW8 = min Cout,
# 0 = off): ResNet tests with it on, same-box config-5 bench A/B and per-layer
# times; plus the host cost of a forward (tools/host_cost_bench.py).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_nw8
mkdir -p $O
timeout -k 10 200 python tools/host_cost_bench.py qdq 256 300 2>&1 | grep -v amdgpu.ids > $O/hc_qdq.txt
cat $O/hc_qdq.txt
timeout -k 10 200 python tools/host_cost_bench.py static 1024 300 2>&1 | grep -v amdgpu.ids > $O/hc_static.txt
cat $O/hc_static.txt
QCN_STREAM_NW8=256 timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for V in 0 256 1024 0 256 1024; do
  QCN_STREAM_NW8=$V timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('QCN_STREAM_NW8=$V: %8.0f img/s  %.3f ms/step' % (d['value'], d['ms_per_step']))"
done
for V in 0 256; do
  QCN_STREAM_NW8=$V timeout -k 10 300 python tools/resnet_layers.py > $O/layers_$V.txt 2>&1
done
paste $O/layers_0.txt $O/layers_256.txt | grep -v amdgpu.ids | awk -F'\t' '{printf "%-92s | %s\n", $1, substr($2,39,8)}' | grep -E "1x1|total"
