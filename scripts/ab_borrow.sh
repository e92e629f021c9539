# A/B of the adds' key handling on whole bench lines (run on the GPU box):
#   bash scripts/ab_borrow.sh CONFIG mode...   (mode: off | large | always, bench.py --borrow)
# Prints ms_per_step, p50/p99, adds and detect per mode; logs in gpurun_out/abb_*.log
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cfg=$1; shift
for rep in $(seq 1 ${REPS:-2}); do
  for m in "$@"; do
    timeout -k 10 400 python -u bench.py --config $cfg --borrow $m --no-cpu --no-shim --lm-batches 0 \
      ${EXTRA:-} > gpurun_out/abb_${cfg}_${m}_$rep.log 2>&1 || { echo "$m failed"; tail -3 gpurun_out/abb_${cfg}_${m}_$rep.log; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('gpurun_out/abb_${cfg}_${m}_$rep.log') if l.startswith('{')][-1])
L=d.get('latency') or {}
print('c$cfg $m rep$rep', 'ms', d['ms_per_step'], 'p50', d['p50_batch_ms'], 'p99', d['p99_batch_ms'], 'adds', d['add_us_mean'],
      'detect', (L.get('detect_us') or {}), 'keys', d['config'].get('keys'))"
  done
done
