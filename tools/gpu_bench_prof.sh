set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu > $R/gpurun_out/prof.log 2>&1
