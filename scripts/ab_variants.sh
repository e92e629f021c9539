# A/B the experiment variants of libfdbcs.so (scripts/build_variants.sh) on the
# HBM-resident bench leg: bash scripts/ab_variants.sh name... (run on the GPU box)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "$@"; do
  FDBCS_LIB_PATH=$PWD/scripts/micro/var/libfdbcs_$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-shim \
    --lm-batches 0 --steps 30 --warmup 5 > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_$v.log; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][-1])
print('$v', d['ms_per_step'], d['p99_batch_ms'], d['hbm_resident']['ms_per_step'], d['roofline']['stage_us'])"
done
