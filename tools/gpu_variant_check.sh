# r05: parity of variant libraries on the headline tests, then a same-box A/B.
# usage (on the box): bash tools/gpu_variant_check.sh TAG LIB_A LIB_B [LIB_C]
# (paths relative to the repo root; the first is the baseline)
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for L in "$@"; do
  QCN_LIB=$R/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests_$(basename $L .so).log 2>&1
  echo "tests-ok $L"
done
ARGS=()
for L in "$@"; do ARGS+=("QCN_LIB=$R/$L"); done
for i in 1 2 3; do
  for E in "${ARGS[@]}"; do
    env $E timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu --no-pmc --no-extra 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('%-40s %9.0f img/s  ' % ('$E'[-40:], d['value']) + ' '.join('%s=%.1f' % (n, v['ms']*1e3) for n, v in k.items()))" | tee -a $O/ab.txt
  done
done
echo done > $O/DONE
