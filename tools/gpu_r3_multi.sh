# r03: GPU tests with the first-K-step correction operand (all conv loops), then
# headline A/B of tools/ab/libqconvnet_b.so (conv_gemm change only) vs _c.so
# (+ the conv3x3 loops), and ResNet a vs c.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_cinit_t.log 2>&1 || { tail -30 gpurun_out/r03_cinit_t.log; exit 1; }
tail -2 gpurun_out/r03_cinit_t.log
bash tools/pair_ab.sh "QCN_LIB=$GRAFT_REPO_ROOT/tools/ab/libqconvnet_b.so" "QCN_LIB=$GRAFT_REPO_ROOT/tools/ab/libqconvnet_c.so" "QCN_LIB=$GRAFT_REPO_ROOT/tools/ab/libqconvnet_b.so" "QCN_LIB=$GRAFT_REPO_ROOT/tools/ab/libqconvnet_c.so"
bash tools/ab_resnet.sh tools/ab/libqconvnet_a.so tools/ab/libqconvnet_c.so 2
