# Round-6 profile set of the bench workload (GPU box): kernel trace + stats of
# the Resolver window with the default (borrowed) batches, and the HBM traffic
# counters in separate passes (FETCH_SIZE, WRITE_SIZE).
#   bash scripts/profile_r06.sh [config=2]
# Outputs: gpurun_out/r06_c<cfg>/{ktrace_summary.txt, kernel_stats.csv, pmc_summary.txt, pmc_traffic.json}
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=${1:-2}
O=gpurun_out/r06_c$cfg
mkdir -p $O
if [ "$cfg" = 5 ]; then ks=6; kw=2; ps=4; pw=1; else ks=200; kw=5; ps=50; pw=5; fi
common="--config $cfg --no-cpu --no-shim --lm-batches 0 --stage-batches 0 --latency-batches 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 -u bench.py $common --steps $ks --warmup $kw > $O/kt.log 2>&1 || { echo "kernel trace failed"; tail -5 $O/kt.log; exit 1; }
kt=$(find $O/kt -name "*kernel_trace.csv" | head -1)
ks_csv=$(find $O/kt -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$kt" $ks k_ingest > $O/ktrace_summary.txt
cp "$ks_csv" $O/kernel_stats.csv
rm -rf $O/kt
echo "kernel trace ok"; head -8 $O/ktrace_summary.txt
for ctr in FETCH_SIZE WRITE_SIZE; do
  FDBCS_LIVE=0 timeout -s KILL 400 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc/p_$ctr -o run -- \
    python3 -u bench.py $common --steps $ps --warmup $pw > $O/pmc_$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -5 $O/pmc_$ctr.log; exit 1; }
  echo "pmc $ctr ok"
done
hp=$(grep -h '^{' $O/pmc_FETCH_SIZE.log | tail -1 | python3 -c "import json,sys; print(json.load(sys.stdin)['config']['history_pre'])")
python3 scripts/pmc_summary.py $O/pmc $ps k_ingest $O/pmc_traffic.json $hp > $O/pmc_summary.txt 2>&1
rm -rf $O/pmc
cat $O/pmc_summary.txt
