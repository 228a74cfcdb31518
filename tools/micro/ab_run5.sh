# conv kernels repeated A/B (tree vs tools/ab/conv3x3_base.hip) + parity + forward timing
set -e
timeout -k 10 400 bash tools/micro/ab_stamp.sh 5 > gpurun_out/ab5.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/par.txt 2>&1
timeout -k 10 120 python -u tools/kbench.py 1024 100 > gpurun_out/kb.txt 2>&1
