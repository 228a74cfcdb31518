# fc1 split-K ablations (diagnostic builds in tools/ab/, results wrong by design)
set -e
mkdir -p gpurun_out/fcab
timeout -k 10 400 bash tools/fc_ab.sh "QCN_DUMMY=0" "QCN_LIB=/root/repo/tools/ab/libfc_NOMFMA.so" "QCN_LIB=/root/repo/tools/ab/libfc_NOSTORE.so" "QCN_DUMMY=0" > gpurun_out/fcabl.txt 2>&1
