# Build a diagnostic variant of libqconvnet.so with classifier.hip compiled
# (r06: the QCN_JOIN_AFF / QCN_FC_U switches this used were removed from csrc/; to rerun, add them back as a patch under tools/patches/.)
# with extra defines (never the product library):
#   bash tools/build_variant_fc.sh NAME "-DQCN_FC_U=8"
set -e
cd "$(dirname "$0")/../convnet-quantization_amd/csrc"
mkdir -p build/var_$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
  -Wall -Wno-unused-function -I../../include -I. $2 -c classifier.hip -o build/var_$1/classifier.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../qconvnet/libqconvnet_$1.so build/conv3x3.o \
  build/elementwise.o build/linear.o build/var_$1/classifier.o build/convgen.o build/convgemm.o build/resnet_qdq.o build/resnet_stem.o
