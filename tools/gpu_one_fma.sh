# conv1's requant in one fma: the headline / W4 / parity GPU tests, then the
# same-process A/B (tools/one_fma_ab.py) at batch 1024 and 256, per-tensor.
# usage (on the box): bash tools/gpu_one_fma.sh TAG
set -e
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_w4.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 300 python tools/one_fma_ab.py 1024 1000 4 2>&1 | grep -v amdgpu | tee $O/ab1024.txt
timeout -k 10 300 python tools/one_fma_ab.py 256 2000 4 2>&1 | grep -v amdgpu | tee $O/ab256.txt
