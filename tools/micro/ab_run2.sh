# classifier head A/B: 256-thread workgroups vs 512 / 1024-thread workgroups (dispatch ramp)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/par.txt 2>&1
mkdir -p gpurun_out/fcab
timeout -k 10 500 bash tools/fc_ab.sh "QCN_FC_BIGWG=0" "QCN_FC_BIGWG=1" "QCN_FC_BIGWG=0" "QCN_FC_BIGWG=1" > gpurun_out/fcab.txt 2>&1
