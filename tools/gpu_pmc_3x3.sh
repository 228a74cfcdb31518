# r03: SQ counters of the ResNet forward per kernel (why the 3x3 convs sit at
# ~30 % of peak): one pass of SQ counters over tools/resnet_layers.py.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_pmc3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA -f csv -d $O/a -o run -- python3 $R/tools/resnet_layers.py > $O/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -f csv -d $O/b -o run -- python3 $R/tools/resnet_layers.py > $O/b.log 2>&1
cd $R
python3 tools/pmc_by_kernel.py $O conv3x3 conv3x3_img conv_gemm_kernel\<256 conv1x1_stream convpair > $O/summary.txt
cat $O/summary.txt
find $O -name '*_agent_info.csv' -delete
