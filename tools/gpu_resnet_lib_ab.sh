# r05: ResNet GPU tests on the product library, then a same-box A/B of the
# ResNet-50 bench across libraries (paths relative to the repo root).
# usage (on the box): bash tools/gpu_resnet_lib_ab.sh TAG LIB_A LIB_B
set -e
TAG=$1; A=$2; B=$3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo tests-ok
for i in 1 2 3; do
  for L in $A $B; do
    QCN_LIB=$R/$L timeout -k 10 300 python bench.py --workload resnet50 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('%-36s %9.0f img/s  %.3f ms/step' % ('$L'[-36:], d['value'], d['ms_per_step']))" | tee -a $O/ab.txt
  done
done
echo done > $O/DONE
