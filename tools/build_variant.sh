# Build a diagnostic variant of libqconvnet.so (never the product library):
#   bash tools/build_variant.sh NAME "-DFOO=1 ..." [PATCH]
# compiles conv3x3.hip with the extra hipcc defines — after applying PATCH
# (a file under tools/patches/, e.g. grid_probe.patch) to a copy of the
# sources in build/var_NAME/ when one is given — and links it with the
# product objects into convnet-quantization_amd/qconvnet/libqconvnet_NAME.so.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT/convnet-quantization_amd/csrc"
mkdir -p build/var_$1
SRC=conv3x3.hip
if [ -n "$3" ]; then
  rm -rf build/var_$1/src && mkdir -p build/var_$1/src
  cp *.hip *.hpp build/var_$1/src/
  (cd build/var_$1/src && patch -s -p3 < "$ROOT/$3")
  SRC=build/var_$1/src/conv3x3.hip
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
  -Wall -Wno-unused-function -I../../include -I. $2 -c $SRC -o build/var_$1/conv3x3.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../qconvnet/libqconvnet_$1.so build/var_$1/conv3x3.o build/convs36.o \
  build/elementwise.o build/linear.o build/classifier.o build/convgen.o build/convgemm.o build/resnet_qdq.o build/resnet_stem.o
