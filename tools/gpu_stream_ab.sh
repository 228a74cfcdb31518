# r03: ResNet GPU tests with the streaming 1x1 kernel at its default (K <= 128)
# and at K <= 256 (weights-resident waves, activations through an LDS ring),
# then a same-box A/B of QCN_GEMM_STREAM on the config-5 bench (two HIP
# streams, as the bench runs it) and single-stream per-layer times.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_stream
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
QCN_GEMM_STREAM=256 timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t256.log 2>&1 || { tail -30 $O/t256.log; exit 1; }
tail -1 $O/t256.log
for S in 0 128 256 0 128 256; do
  QCN_GEMM_STREAM=$S timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('stream=$S %8.0f img/s  %.3f ms/step' % (d['value'], d['ms_per_step']))"
done
for S in 128 256; do
  QCN_GEMM_STREAM=$S timeout -k 10 300 python tools/resnet_layers.py > $O/layers_$S.txt 2>&1
done
paste $O/layers_128.txt $O/layers_256.txt | grep -v amdgpu.ids | awk -F'\t' '{printf "%-92s | %s\n", $1, substr($2,39,8)}'
