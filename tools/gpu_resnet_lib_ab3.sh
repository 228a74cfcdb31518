# r05: same-box A/B of the ResNet-50 bench across three libraries (no tests).
# usage (on the box): bash tools/gpu_resnet_lib_ab3.sh TAG LIB_A LIB_B LIB_C
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for i in 1 2 3; do
  for L in "$@"; do
    QCN_LIB=$R/$L timeout -k 10 300 python bench.py --workload resnet50 --no-cpu --no-pmc 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('%-36s %9.0f img/s  %.3f ms/step' % ('$L'[-36:], d['value'], d['ms_per_step']))" | tee -a $O/ab.txt
  done
done
echo done > $O/DONE
