# Kernel trace of the bench's Resolver window with borrowed batches (run on the GPU box):
#   bash scripts/profile_borrow.sh [config=2] [borrow=always]
# Outputs: gpurun_out/pb_c<cfg>/ktrace_summary.txt, timeline.txt (three batches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=${1:-2}; bm=${2:-always}
O=gpurun_out/pb_c${cfg}_$bm
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 -u bench.py --config $cfg --borrow $bm --no-cpu --no-shim --lm-batches 0 --stage-batches 0 \
  --latency-batches 0 --steps ${STEPS:-100} --warmup 5 > $O/kt.log 2>&1 || { echo "kernel trace failed"; tail -5 $O/kt.log; exit 1; }
kt=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_summary.py "$kt" ${STEPS:-100} ${MARK:-k_ingest} > $O/ktrace_summary.txt
d=$(dirname $kt); cp $kt $d/run_kernel_trace.csv 2>/dev/null
for w in -4 -3 -2; do echo "== batch $w"; python3 scripts/timeline.py $d ${MARK:-k_ingest} $w; done > $O/timeline.txt
rm -rf $O/kt
head -20 $O/ktrace_summary.txt; head -40 $O/timeline.txt
