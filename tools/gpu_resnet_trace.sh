# r05: rocprofv3 kernel-trace stats of the ResNet-50 bench command (configs[4]).
# usage (on the box): bash tools/gpu_resnet_trace.sh TAG
set -e
TAG=${1:-rtrace}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/t -o run -- python3 $R/bench.py --workload resnet50 --no-cpu --no-pmc --steps 20 --warmup 5 > $O/trace.log 2>&1
cd $R
cp $O/t/run_kernel_stats.csv $O/kernel_stats.csv
find $O -name '*_kernel_trace.csv' -delete
find $O -name '*_agent_info.csv' -delete
echo done > $O/DONE
