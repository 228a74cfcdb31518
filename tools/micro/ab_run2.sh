# classifier head A/B: K-quarter XCD map vs row-block map + XCD-local finisher rows
set -e
QCN_FC_LOCAL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "classifier or full_net" > gpurun_out/par.txt 2>&1
mkdir -p gpurun_out/fcab
timeout -k 10 500 bash tools/fc_ab.sh "QCN_FC_LOCAL=0" "QCN_FC_LOCAL=1" "QCN_FC_LOCAL=0" "QCN_FC_LOCAL=1" > gpurun_out/fcab.txt 2>&1
