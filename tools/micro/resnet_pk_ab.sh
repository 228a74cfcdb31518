set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/rn_par.txt 2>&1
for L in "" "QCN_LIB=tools/ab/libqconvnet_pk.so" "" "QCN_LIB=tools/ab/libqconvnet_pk.so"; do
  echo "== [$L]"
  env $L timeout -k 10 300 python bench.py --workload resnet50 --no-cpu --steps 10 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['roofline']['achieved'])"
done
