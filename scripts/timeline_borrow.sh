# Device timeline of borrowed batches (kernels + copies; run on the GPU box):
#   bash scripts/timeline_borrow.sh [config=2]   (env passes through, e.g. FDBCS_INGEST_OVERLAP=0)
# Outputs: gpurun_out/tl_c<cfg>/timeline.txt (four staged batches of the timed region)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=${1:-2}
O=gpurun_out/tl_c${cfg}${TAG:-}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/kt -o run -- \
  python3 -u bench.py --config $cfg --borrow always --no-cpu --no-shim --lm-batches 0 --stage-batches 0 \
  --latency-batches 0 --steps ${STEPS:-60} --warmup 5 > $O/kt.log 2>&1 || { echo "trace failed"; tail -5 $O/kt.log; exit 1; }
kt=$(find $O/kt -name "*kernel_trace.csv" | head -1)
d=$(dirname $kt); cp $kt $d/run_kernel_trace.csv
mc=$(find $O/kt -name "*memory_copy_trace.csv" | head -1); [ -n "$mc" ] && cp $mc $d/run_memory_copy_trace.csv
for w in -8 -6 -4 -2; do echo "== staged batch $w"; python3 scripts/timeline.py $d k_ingest_staged $w; done > $O/timeline.txt
rm -rf $O/kt
head -60 $O/timeline.txt
