# r05: config 2 with conv5+6 as the separate cout-split launch — parity
# (headline + models tests), then a same-box A/B against libqconvnet_sm1.so.
set -e
TAG=${1:-sm}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_models.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 bash tools/ab.sh "" "QCN_LIB=$R/convnet-quantization_amd/qconvnet/libqconvnet_sm1.so" 3 "--workload qdq" > $O/ab.txt 2>&1
cat $O/ab.txt
