# r06 pass 1 (on the box): full GPU tests on the product library, then a
# same-box A/B of the product against the r05 conv3x3 (libqconvnet_r05.so:
# the r05 one-launch kernel with its spills) on the headline bench, then the
# clock probe (per-phase and per-layer table).
set -o pipefail
O=gpurun_out
L=convnet-quantization_amd/qconvnet
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/r06_p1_gpu_tests.log 2>&1 || { echo "tests failed rc=$?" >> $O/r06_p1_gpu_tests.log; exit 1; }
for r in 1 2; do
  for v in prod r05; do
    if [ $v = prod ]; then lib=$L/libqconvnet.so; else lib=$L/libqconvnet_$v.so; fi
    echo "## $v round $r" >> $O/r06_p1_ab.txt
    QCN_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-pmc --no-extra --steps 400 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(round(d['value']/1e6,4), 'M img/s', round(d['ms_per_step']*1e3,2), 'us/step', {k: v['ms']*1e3 for k, v in d['kernels'].items()})" >> $O/r06_p1_ab.txt || exit 1
  done
done
if [ -f tools/clock/libqconvnet_clock.so ]; then
  timeout -k 10 200 python -u tools/clock_probe.py --batch 1024 > $O/r06_p1_clock.txt 2>&1 || exit 1
fi
timeout -k 10 300 python -u tools/w4_ab.py 1024 500 3 > $O/r06_p1_w4_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/c16_ab.py 1024 500 3 > $O/r06_p1_c16_ab.txt 2>&1 || exit 1
