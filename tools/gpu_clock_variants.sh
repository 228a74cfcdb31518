# Diagnostic: tools/clock_probe.py under several stamped libraries (paths
# relative to the repo root), one after the other on the same box.
# usage (on the box): bash tools/gpu_clock_variants.sh TAG LIB...
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for L in "$@"; do
  N=$(basename $L .so)
  QCN_CLOCK_LIB=$R/$L timeout -k 10 200 python tools/clock_probe.py > $O/$N.json 2> $O/$N.txt
  echo "== $N"; grep "#" $O/$N.txt
done
