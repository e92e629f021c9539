# Stage timings for library variants (scripts/micro/var/*.so), same workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in scripts/micro/var/*.so; do
  FDBCS_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --warmup ${WARM:-2500} --steps 100 --stage-batches 30 --no-cpu > gpurun_out/var.log 2>gpurun_out/var.err || { echo "$lib failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/var.log')); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r['batch_us'], r['stage_us'])" $lib
done
