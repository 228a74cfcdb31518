# End-of-milestone GPU pass: all GPU tests + smoke, the three bench lines
# (headline with PMC / clock / CPU baselines, config 2, config 5), and the
# rocprofv3 kernel-trace stats of the headline bench command itself and of
# tools/kbench.py.
# usage (on the box): bash tools/gpu_round_pass.sh TAG
set -e
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --no-cpu --no-pmc --pipeline 2 > $O/bench_pipe2.json 2> $O/bench_pipe2.err
timeout -k 10 300 python bench.py --workload qdq > $O/bench_qdq.json 2> $O/bench_qdq.err
timeout -k 10 400 python bench.py --workload resnet50 > $O/bench_resnet.json 2> $O/bench_resnet.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/tools/kbench.py 1024 100 > $O/trace.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/btrace -o run -- python3 $R/bench.py --no-cpu --steps 50 --warmup 10 > $O/btrace.log 2>&1
cd $R
cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || true
cp $O/btrace/run_kernel_stats.csv $O/bench_kernel_stats.csv 2>/dev/null || true
find $O -name '*_kernel_trace.csv' -delete
find $O -name '*_agent_info.csv' -delete
echo done > $O/DONE
