# A/B library variants (scripts/build_variants.sh) on a bench config:
#   bash scripts/ab_libs.sh CONFIG name...   (run on the GPU box)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cfg=$1; shift
for v in "$@"; do
  FDBCS_LIB_PATH=$PWD/scripts/micro/var/libfdbcs_$v.so timeout -k 10 200 python -u bench.py --config $cfg --no-cpu \
    --no-shim --lm-batches 0 --steps ${STEPS:-30} --warmup ${WARMUP:-5} > gpurun_out/ab_${cfg}_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_${cfg}_$v.log; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_${cfg}_$v.log') if l.startswith('{')][-1])
print('c$cfg $v', d['ms_per_step'], d['p50_batch_ms'], d['hbm_resident']['ms_per_step'], d['roofline']['stage_us'])"
done
