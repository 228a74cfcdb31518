# Per-layer ResNet-50 times (tools/resnet_layers.py) for the tree's library.
set -e
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python tools/resnet_layers.py > $O/layers.txt 2>&1
