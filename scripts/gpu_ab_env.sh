# A/B of an environment switch on one box: bench stage timings with VAR unset / set, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAR=$1
for k in 1 2; do
  for mode in off on; do
    if [ $mode = on ]; then export $VAR=1; else unset $VAR; fi
    timeout -k 10 200 python -u bench.py --warmup ${WARM:-2500} --steps 300 --stage-batches 50 --no-cpu > gpurun_out/ab.log 2>gpurun_out/ab.err || { echo "$mode failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.log')); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r['batch_us'], r['stage_us'])" "$VAR=$mode"
  done
done
