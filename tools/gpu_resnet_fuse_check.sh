# r05: the ResNet GPU tests (fused layer-1 reduce included), then a same-box
# A/B of the ResNet-50 bench with the reduce fused vs separate launches.
# usage (on the box): bash tools/gpu_resnet_fuse_check.sh TAG
set -e
TAG=${1:-resfuse}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo tests-ok
for i in 1 2 3; do
  for F in "" "--separate-reduce"; do
    timeout -k 10 300 python bench.py --workload resnet50 --no-cpu --no-pmc $F 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('%-20s %9.0f img/s  %.3f ms/step' % ('[$F]', d['value'], d['ms_per_step']))" | tee -a $O/ab.txt
  done
done
echo done > $O/DONE
