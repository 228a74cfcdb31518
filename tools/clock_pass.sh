# Effective clock per kernel (MICROARCH 'DVFS give-back': GRBM_GUI_ACTIVE / 8 /
# kernel wall) plus MFMA / VALU busy, at a batch large enough that each
# dispatch is >= 0.3 ms.  usage (on the box): bash tools/clock_pass.sh TAG [B]
set -e
TAG=${1:-clock}; B=${2:-8192}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/kbench.py $B 20 > $O/kbench.txt 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES -f csv -d $O/pmc -o run -- python3 $R/tools/kbench.py $B 10 > $O/pmc.log 2>&1
cd $R
python3 tools/clock_summary.py $O/pmc > $O/clock_summary.txt 2>&1 || true
find $O -name '*_counter_collection.csv' -size +20M -delete
echo done > $O/DONE
