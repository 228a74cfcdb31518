# v16 perf pass (parity gate, bench line, rocprof kernel trace + PMC)
set -e
timeout -k 10 1000 bash tools/gpu_perf.sh v16
