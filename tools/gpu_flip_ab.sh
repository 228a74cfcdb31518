# r03: in-ring u8->s8 flip in the streaming 1x1 (each wave flips the pieces it
# DMA'd once, instead of every wave flipping every B fragment it reads).
# ResNet GPU tests on the new library, then same-box A/B of config 5 and the
# single-stream layer times.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_flip
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 600 bash tools/ab_resnet.sh tools/ab/lib_base.so tools/ab/lib_flip.so 3
for L in base flip; do
  QCN_LIB=tools/ab/lib_$L.so timeout -k 10 300 python tools/resnet_layers.py > $O/layers_$L.txt 2>&1
done
paste -d'|' <(grep "conv 1x1" $O/layers_base.txt | cut -c1-60) <(grep "conv 1x1" $O/layers_flip.txt | cut -c50-60)
tail -1 $O/layers_base.txt $O/layers_flip.txt
