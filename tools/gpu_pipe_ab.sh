# r03: parity of the persistent prefetching conv3+4 (QCN_PAIR34=22), then
# same-box A/B against the ring pair (0) and the weights-from-L2 pair (2).
set -e
cd $GRAFT_REPO_ROOT
QCN_PAIR34=22 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pair or headline or conv56 or qdq" > gpurun_out/r03_pipe_t.log 2>&1 || { tail -40 gpurun_out/r03_pipe_t.log; exit 1; }
tail -2 gpurun_out/r03_pipe_t.log
bash tools/pair_ab.sh "QCN_PAIR34=0" "QCN_PAIR34=22" "QCN_PAIR34=2" "QCN_PAIR34=0" "QCN_PAIR34=22"
