# GPU perf pass: parity gate, the default bench line (with CPU baselines), kernel
# trace of the same command, PMC counters (separate passes, as the guide says).
# usage (on the box, from the repo root): bash tools/gpu_perf.sh TAG
set -e
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu --no-pmc > $O/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -f csv -d $O/pmc_sq -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-pmc > $O/pmc_sq.log 2>&1 || echo "pmc_sq failed" >> $O/errors.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-pmc > $O/pmc_fetch.log 2>&1 || echo "pmc_fetch failed" >> $O/errors.txt
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-pmc > $O/pmc_write.log 2>&1 || echo "pmc_write failed" >> $O/errors.txt

# keep the summaries, drop the per-dispatch csvs (they overflow gpurun_out's 64 MiB)
cd $R
python tools/pmc_summary.py $O > $O/pmc_summary.txt 2>&1 || true
cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || true
find $O -name '*_counter_collection.csv' -delete
find $O -name '*_kernel_trace.csv' -delete
find $O -name '*_agent_info.csv' -delete
du -sh $O > $O/du.txt
echo done > $O/DONE
