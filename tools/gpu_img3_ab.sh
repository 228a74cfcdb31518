# r03: whole-image 3x3 kernel for the 14x14x256 / 7x7x512 maps (QCN_GEMM_IMG3
# 0 = tiled, 1 = 14x14 maps, 2 = also 7x7x512): tests, same-box config-5 bench
# A/B and per-layer times.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_img3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
QCN_GEMM_IMG3=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread -k "whole_image or bit_exact" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
for V in 0 1 2 0 1 2; do
  QCN_GEMM_IMG3=$V timeout -k 10 300 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('QCN_GEMM_IMG3=$V: %8.0f img/s  %.3f ms/step' % (d['value'], d['ms_per_step']))"
done
for V in 0 1 2; do
  QCN_GEMM_IMG3=$V timeout -k 10 300 python tools/resnet_layers.py > $O/layers_$V.txt 2>&1
done
paste $O/layers_0.txt $O/layers_1.txt $O/layers_2.txt | grep -v amdgpu.ids | awk -F'\t' '{printf "%-92s | %s | %s\n", $1, substr($2,39,8), substr($3,39,8)}' | grep -E "3x3    1   (14|7) |total"
