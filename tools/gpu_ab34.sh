# conv3+conv4 launch forms, same process, per library variant.
# usage: bash tools/gpu_ab34.sh TAG "variant ..." [B]   (variant "" = the product library)
set -e
O=gpurun_out/$1
mkdir -p $O
for v in $2; do
  if [ "$v" = "prod" ]; then lib=convnet-quantization_amd/qconvnet/libqconvnet.so; else lib=convnet-quantization_amd/qconvnet/libqconvnet_$v.so; fi
  echo "== $v" >> $O/ab.txt
  QCN_LIB=$PWD/$lib timeout -k 10 120 python3 tools/conv34_ab.py ${3:-1024} 200 5 >> $O/ab.txt 2>&1
done
