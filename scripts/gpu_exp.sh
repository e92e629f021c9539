# Stage timings under FDBCS_EXP experiment modes (results invalid for modes != 0).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in "$@"; do
  FDBCS_EXP=$m timeout -k 10 200 python -u bench.py --warmup ${WARM:-2500} --steps 100 --stage-batches 30 --no-cpu > gpurun_out/exp.log 2>gpurun_out/exp.err || { echo "mode $m failed"; tail -5 gpurun_out/exp.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/exp.log')); r=d['roofline']; print('mode', sys.argv[1], d['ms_per_step'], r['batch_us'], r['stage_us'])" $m
done
