# PMC passes over tools/resnet_layers.py (run on the GPU box from the repo root)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_rn
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY -f csv -d $O/sq -o run -- python3 $R/tools/resnet_layers.py > $O/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -f csv -d $O/mem -o run -- python3 $R/tools/resnet_layers.py > $O/mem.log 2>&1 || echo "mem pass failed" >> $O/errors.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/tools/resnet_layers.py > $O/trace.log 2>&1
