# Config-5 kernel trace of the HBM-resident batches (run on the GPU box):
#   bash scripts/profile_c5.sh [extra env assignments are inherited]
# Summary: gpurun_out/c5kt/summary.txt (the last 3 batches by k_ingest markers)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c5kt
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 -u bench.py --config 5 --no-cpu --no-shim --lm-batches 0 --steps 2 --warmup 1 --stage-batches 4 > $O/kt.log 2>&1 \
  || { echo "kernel trace failed"; tail -5 $O/kt.log; exit 1; }
kt=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_summary.py "$kt" 3 "k_ingest<" > $O/summary.txt 2>&1
rm -rf $O/kt
head -40 $O/summary.txt
