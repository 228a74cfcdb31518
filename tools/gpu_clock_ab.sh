# Per-phase cycles / clock of the one-launch convs, two stamped libraries
# alternating (tools/clock_probe.py): bash tools/gpu_clock_ab.sh TAG LIB_A LIB_B [N]
set -e
TAG=$1; A=$2; B=$3; N=${4:-2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for i in $(seq $N); do
  for L in $A $B; do
    echo "== $L" >> $O/clock.txt
    QCN_CLOCK_LIB=$R/$L timeout -k 10 200 python tools/clock_probe.py > $O/probe.json 2>> $O/clock.txt
  done
done
cat $O/clock.txt
