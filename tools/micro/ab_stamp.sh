# Same-box A/B of the conv kernels through conv_stamp.hip: the tree's
# conv3x3.hip against tools/ab/conv3x3_base.hip (e.g. `git show HEAD:...`).
# usage (on the box, from the repo root): bash tools/micro/ab_stamp.sh [reps]
set -e
N=${1:-2}
B=/tmp/abbase
mkdir -p $B/convnet-quantization_amd/csrc $B/tools/micro
cp convnet-quantization_amd/csrc/*.hpp $B/convnet-quantization_amd/csrc/
cp tools/ab/conv3x3_base.hip $B/convnet-quantization_amd/csrc/conv3x3.hip
cp tools/micro/conv_stamp.hip $B/tools/micro/
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS -Iinclude"
hipcc $F -I$B/convnet-quantization_amd/csrc $B/tools/micro/conv_stamp.hip -o /tmp/stamp_base
hipcc $F -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/stamp_new
for i in $(seq $N); do
  echo "=== base"; timeout -k 10 60 /tmp/stamp_base | grep "us/launch"
  echo "=== new";  timeout -k 10 60 /tmp/stamp_new | grep "us/launch"
done
