# Round-5 profile set of the bench workload (run on the GPU box):
#   kernel trace + stats of the per-transaction window (live ingest),
#   the host/device timeline of the window, and the HBM traffic counters.
#   bash scripts/profile_r05.sh [config=2]
# Outputs under gpurun_out/r05/ (summaries copied to profiles/ by hand).
# PMC passes run with FDBCS_LIVE=0: counter collection serializes dispatches,
# and a live kernel waits for adds that a blocked host would never make.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=${1:-2}
O=gpurun_out/r05_c$cfg
mkdir -p $O
common="--config $cfg --no-cpu --no-shim --lm-batches 0 --stage-batches 0 --latency-batches 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 -u bench.py $common --steps 200 --warmup 5 > $O/kt.log 2>&1 || { echo "kernel trace failed"; tail -5 $O/kt.log; exit 1; }
kt=$(find $O/kt -name "*kernel_trace.csv" | head -1)
ks=$(find $O/kt -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$kt" 200 k_live_ingest > $O/ktrace_summary.txt
cp "$ks" $O/kernel_stats.csv
rm -rf $O/kt
echo "kernel trace ok"
FDBWL_MARK=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d $O/api -- \
  python3 -u bench.py $common --steps 40 --warmup 5 > $O/api.log 2>&1 || { echo "api trace failed"; tail -5 $O/api.log; exit 1; }
python3 scripts/api_timeline.py $O/api 30 2 > $O/api_timeline.txt 2>&1
rm -rf $O/api
echo "api timeline ok"
for ctr in FETCH_SIZE WRITE_SIZE; do
  FDBCS_LIVE=0 timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc/p_$ctr -o run -- \
    python3 -u bench.py $common --steps 50 --warmup 5 > $O/pmc_$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -5 $O/pmc_$ctr.log; exit 1; }
  echo "pmc $ctr ok"
done
python3 scripts/pmc_summary.py $O/pmc 49 k_ingest > $O/pmc_summary.txt 2>&1
echo done
