# r05: the 16x16x64 pair phases — parity on the headline / pair tests, then a
# same-box A/B against the 32x32x32 build (libqconvnet_m32.so, QCN_M16=0).
# usage (on the box): bash tools/gpu_m16_check.sh TAG
set -e
TAG=${1:-m16}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo tests-ok
timeout -k 10 500 bash tools/ab.sh "" "QCN_LIB=$R/convnet-quantization_amd/qconvnet/libqconvnet_m32.so" 3 > $O/ab.txt 2>&1
cat $O/ab.txt
echo done > $O/DONE
