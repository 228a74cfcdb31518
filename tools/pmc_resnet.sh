# PMC passes over tools/resnet_layers.py (run on the GPU box from the repo
# root), one counter group per pass (FETCH_SIZE and WRITE_SIZE together would
# exceed the 4 TCC counters of one pass).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pmc_rn}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY -f csv -d $O/sq -o run -- python3 $R/tools/resnet_layers.py > $O/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 $R/tools/resnet_layers.py > $O/fetch.log 2>&1 || echo "fetch pass failed" >> $O/errors.txt
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -f csv -d $O/write -o run -- python3 $R/tools/resnet_layers.py > $O/write.log 2>&1 || echo "write pass failed" >> $O/errors.txt
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 $R/tools/resnet_layers.py > $O/trace.log 2>&1
cd $R
python3 tools/pmc_resnet_summary.py $O > $O/summary.txt 2>&1 || true
find $O -name '*_agent_info.csv' -delete
