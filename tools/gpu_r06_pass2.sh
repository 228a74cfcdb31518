# r06 pass 2 (on the box): clock probe (per-phase + per-layer table), the W4
# two-launch and the three-launch same-process A/Bs against the one launch
set -o pipefail
O=gpurun_out
timeout -k 10 200 python -u tools/clock_probe.py --batch 1024 > $O/r06_p2_clock.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/w4_ab.py 1024 500 3 > $O/r06_p2_w4_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/c16_ab.py 1024 500 3 > $O/r06_p2_c16_ab.txt 2>&1 || exit 1
