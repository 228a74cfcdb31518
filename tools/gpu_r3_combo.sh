# r03: full GPU tests at the tree's library (first-K-step correction operand +
# 128-pixel thin-conv tiles), the headline A/B of the correction operand
# (tools/ab/libqconvnet_b.so vs _c.so), then the thin-tile A/B (env).
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_combo_t.log 2>&1 || { tail -30 gpurun_out/r03_combo_t.log; exit 1; }
tail -2 gpurun_out/r03_combo_t.log
bash tools/pair_ab.sh "QCN_LIB=$GRAFT_REPO_ROOT/tools/ab/libqconvnet_b.so" "QCN_LIB=$GRAFT_REPO_ROOT/tools/ab/libqconvnet_c.so" "QCN_LIB=$GRAFT_REPO_ROOT/tools/ab/libqconvnet_b.so" "QCN_LIB=$GRAFT_REPO_ROOT/tools/ab/libqconvnet_c.so"
bash tools/gpu_thin_ab.sh
