set -e
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS -Iinclude -Iconvnet-quantization_amd/csrc"
for P in 0 1 2 3; do hipcc $F -DQCN_PROD_PRIO=$P tools/micro/conv_stamp.hip -o /tmp/st_$P & done; wait
for r in 1 2 3; do for P in 0 1 2 3; do echo "prio $P: $(timeout -k 10 60 /tmp/st_$P | grep conv12)"; done; done
