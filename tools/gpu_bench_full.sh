# The driver's default bench command (all fields: PMC passes, clock / phase
# table, CPU baselines, configs_extra children), then its own rocprofv3
# kernel-trace stats.  usage (on the box): bash tools/gpu_bench_full.sh TAG
set -e
TAG=${1:-full}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err
echo bench-ok
cat $O/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline'].get('frac'), list(d.get('configs_extra',{}).keys()))"
echo done > $O/DONE
