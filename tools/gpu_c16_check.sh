# One-launch conv1..conv6 check on the box: its parity tests and the headline /
# pair tests, then a forward timing A/B (tools/kbench.py with and without it).
# usage (on the box): bash tools/gpu_c16_check.sh TAG
set -e
O=gpurun_out/${1:-c16}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "one_launch or headline or pair or config2" --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python tools/c16_ab.py > $O/ab.txt 2>&1
