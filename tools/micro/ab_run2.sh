# fc1 split-K A/B: 4 waves vs 8 waves (K quarter halved inside the workgroup)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/par.txt 2>&1
mkdir -p gpurun_out/fcab
timeout -k 10 500 bash tools/fc_ab.sh "QCN_FC_KH=1" "QCN_FC_KH=2" "QCN_FC_KH=1" "QCN_FC_KH=2" > gpurun_out/fcab.txt 2>&1
