# r05 diagnostic: L2 hit/miss and HBM requests of the headline's kernels
# (tools/kbench.py batch 1024), one counter set per rocprofv3 pass.
# usage (on the box): bash tools/gpu_pmc_l2.sh TAG [QCN_LIB path]
set -e
TAG=${1:-pmc_l2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
[ -n "$2" ] && export QCN_LIB=$R/$2
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -f csv -d $O/a -o run -- python3 $R/tools/kbench.py 1024 20 > $O/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/b -o run -- python3 $R/tools/kbench.py 1024 20 > $O/b.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCP_TCC_READ_REQ_sum -f csv -d $O/c -o run -- python3 $R/tools/kbench.py 1024 20 > $O/c.log 2>&1
cd $R
python3 tools/pmc_by_kernel.py $O convnet_convs16 fc_splitk fc_finish > $O/summary.txt
cat $O/summary.txt
find $O -name '*_kernel_trace.csv' -delete
find $O -name '*_agent_info.csv' -delete
