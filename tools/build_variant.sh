# Build a diagnostic variant of libqconvnet.so with extra hipcc defines (never
# the product library): bash tools/build_variant.sh NAME "-DFOO=1 ..."
set -e
cd "$(dirname "$0")/../convnet-quantization_amd/csrc"
mkdir -p build/var_$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
  -Wall -Wno-unused-function -I../../include -I. $2 -c conv3x3.hip -o build/var_$1/conv3x3.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../qconvnet/libqconvnet_$1.so build/var_$1/conv3x3.o build/convs36.o \
  build/elementwise.o build/linear.o build/classifier.o build/convgen.o build/convgemm.o build/resnet_qdq.o build/resnet_stem.o
