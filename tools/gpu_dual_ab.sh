# r03: parity of the dual-half pair kernels, then same-box A/B of the pair forms.
set -e
R=$GRAFT_REPO_ROOT
cd $R
QCN_PAIR34=12 QCN_PAIR56=13 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pair or headline or conv56" > gpurun_out/r03_dual_t.log 2>&1 || { tail -30 gpurun_out/r03_dual_t.log; exit 1; }
tail -2 gpurun_out/r03_dual_t.log
bash tools/pair_ab.sh "$@"
