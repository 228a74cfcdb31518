# r03: why the streaming 1x1 conv is slow — access-shape micro probe, the
# single-conv probe for both kernels, and PMC passes over the probe.
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r03_sdiag
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/stream_shape tools/micro/stream_shape.hip
timeout -k 10 120 /tmp/stream_shape | tee $O/shape.txt
for S in 0 1; do
  for R in 1 0; do
    QCN_GEMM_STREAM=$S RESID=$R timeout -k 10 120 python tools/conv1x1_probe.py | tee -a $O/probe.txt
  done
done
cd /tmp && export TMPDIR=/tmp
for S in 0 1; do
  QCN_GEMM_STREAM=$S timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/f$S -o run -- python3 $GRAFT_REPO_ROOT/tools/conv1x1_probe.py > $O/f$S.log 2>&1
  QCN_GEMM_STREAM=$S timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/w$S -o run -- python3 $GRAFT_REPO_ROOT/tools/conv1x1_probe.py > $O/w$S.log 2>&1
  QCN_GEMM_STREAM=$S timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM -f csv -d $O/s$S -o run -- python3 $GRAFT_REPO_ROOT/tools/conv1x1_probe.py > $O/s$S.log 2>&1
  QCN_GEMM_STREAM=$S timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -f csv -d $O/t$S -o run -- python3 $GRAFT_REPO_ROOT/tools/conv1x1_probe.py > $O/t$S.log 2>&1 || echo "ta pass failed $S"
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r03_sdiag"
for S in "01":
    tot = {}
    for tag in "fwst":
        for f in glob.glob(f"{O}/{tag}{S}/**/*counter_collection.csv", recursive=True):
            per = {}
            for r in csv.DictReader(open(f)):
                if "conv" not in r["Kernel_Name"]:
                    continue
                k = (int(r["Dispatch_Id"]), r["Counter_Name"])
                per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
            ids = sorted({k[0] for k in per})[-40:]
            for (i, c), val in per.items():
                if i in ids:
                    tot.setdefault(c, []).append(val)
    print(f"QCN_GEMM_STREAM={S}: " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(tot.items())))
PY
find $O -name '*_agent_info.csv' -delete
