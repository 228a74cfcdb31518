# fc1 split-K tile-to-XCD map A/B (row-block-major vs K-quarter-major) + GPU parity
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/par.txt 2>&1
mkdir -p gpurun_out/fcab
timeout -k 10 400 bash tools/fc_ab.sh "QCN_FC_KMAP=0" "QCN_FC_KMAP=1" "QCN_FC_KMAP=0" "QCN_FC_KMAP=1" > gpurun_out/fcab.txt 2>&1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for V in 0 1; do
  QCN_FC_KMAP=$V timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/fcpmc$V -o run -- python3 $R/tools/kbench.py 1024 20 > $R/gpurun_out/fcpmc$V.log 2>&1
done
cd $R && python3 - <<'PY' > gpurun_out/fcpmc.txt
import csv, glob, collections
for v in (0, 1):
    f = glob.glob(f"gpurun_out/fcpmc{v}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "fc_" in r["Kernel_Name"]:
            acc[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
    for k, xs in acc.items():
        print(v, k, "FETCH_SIZE KB avg", sum(xs) / len(xs))
PY
find gpurun_out -name '*counter_collection.csv' -delete
