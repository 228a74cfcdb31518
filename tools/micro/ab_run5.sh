# conv12-only repeated A/B (tree vs tools/ab/conv3x3_base.hip)
set -e
timeout -k 10 400 bash tools/micro/ab_stamp.sh 8 > gpurun_out/ab5.txt 2>&1
