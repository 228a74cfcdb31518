# Diagnostic library (never the product): the product objects with the
# conv3..conv6 launch replaced by its stamped build (-DQCN_W4_STAMP):
# convnet-quantization_amd/qconvnet/libqconvnet_w4stamp.so, read by tools/w4_stamps.py
set -e
cd "$(dirname "$0")/../convnet-quantization_amd/csrc"
mkdir -p build/var_w4stamp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
  -Wall -Wno-unused-function -I../../include -I. -DQCN_W4_STAMP $1 -c convs36.hip -o build/var_w4stamp/convs36.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../qconvnet/libqconvnet_w4stamp.so build/conv3x3.o \
  build/var_w4stamp/convs36.o build/elementwise.o build/linear.o build/classifier.o build/convgen.o build/convgemm.o \
  build/resnet_qdq.o build/resnet_stem.o
