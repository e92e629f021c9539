# Config-5 A/B of library variants by the HBM-resident batch and stage times
# (run on the GPU box): bash scripts/ab_c5.sh name...   ("base": the product library)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abc5
for v in "$@"; do
  if [ "$v" = base ]; then unset FDBCS_LIB_PATH; else export FDBCS_LIB_PATH=$PWD/scripts/micro/var/libfdbcs_$v.so; fi
  timeout -k 10 400 python3 -u bench.py --config 5 --no-cpu --no-shim --lm-batches 0 --steps 2 --warmup 1 --stage-batches 4 \
    > gpurun_out/abc5/$v.json 2> gpurun_out/abc5/$v.err || { echo "$v failed"; tail -3 gpurun_out/abc5/$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/abc5/$v.json').read().strip().splitlines()[-1])
print('$v', d['hbm_resident']['ms_per_step'], d['roofline'].get('stage_us'))"
done
