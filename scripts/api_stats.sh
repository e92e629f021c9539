# HIP API call counts and time per batch of the bench's Resolver window (GPU box):
#   bash scripts/api_stats.sh [config=2]
# Outputs: gpurun_out/api_c<cfg>/hip_api_stats.csv (+ a per-batch summary on stdout)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=${1:-2}
O=gpurun_out/api_c$cfg
mkdir -p $O
timeout -k 10 300 rocprofv3 --hip-trace --stats --output-format csv -d $O/t -o run -- \
  python3 -u bench.py --config $cfg --borrow always --no-cpu --no-shim --lm-batches 0 --stage-batches 0 \
  --latency-batches 0 --steps ${STEPS:-200} --warmup 5 > $O/run.log 2>&1 || { echo "trace failed"; tail -5 $O/run.log; exit 1; }
st=$(find $O/t -name "*hip_api_stats.csv" | head -1)
cp "$st" $O/hip_api_stats.csv
rm -rf $O/t
python3 -c "
import csv
rows = list(csv.DictReader(open('$O/hip_api_stats.csv')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:25]:
    print('%-34s %9s calls %12.1f us total %9.2f us avg' % (r['Name'][:34], r['Calls'], float(r['TotalDurationNs']) / 1e3, float(r['AverageNs']) / 1e3))
"
