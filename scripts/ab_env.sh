# A/B environment knobs on the bench (per-transaction window + HBM-resident leg):
#   bash scripts/ab_env.sh "name:VAR=1 VAR2=x" "base:" ...   (run on the GPU box)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python -u bench.py --config ${CONFIG:-2} --no-cpu --no-shim --lm-batches 0 --steps ${STEPS:-30} --warmup 5 \
    > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -3 gpurun_out/ab_$name.log; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_$name.log') if l.startswith('{')][-1])
print('$name', d['ms_per_step'], d['p50_batch_ms'], d['p99_batch_ms'], d['add_us_mean'], d['hbm_resident']['ms_per_step'], d['roofline']['stage_us'])"
done
