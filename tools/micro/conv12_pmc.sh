# Effective clock and issue counters of conv12 and the pair kernels under
# ablation builds (diagnostic: outputs wrong by design for the ablations).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c12pmc; mkdir -p $O
for V in "" "-DQCN_EXP_NOCONS" "-DQCN_EXP_NOPROD"; do
  T=$(echo "x$V" | tr -d ' =-')
  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -DQCN_STAMPS $V -Iinclude -Iconvnet-quantization_amd/csrc tools/micro/conv_stamp.hip -o /tmp/cs_$T
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -f csv -d $O/$T -o run -- /tmp/cs_$T > $O/$T.log 2>&1)
  echo "=== $V"
  python3 tools/clock_summary.py $O/$T
  find $O/$T -name '*.csv' -size +5M -delete
done
