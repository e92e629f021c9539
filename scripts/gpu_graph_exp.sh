# Experiment: graph replay vs stream launches (timing only; bench warmup through detect_view, timed steps through detect_device)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in scripts/micro/var/*.so; do
  FDBCS_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --warmup 1500 --steps 200 --stage-batches 0 --pcie-batches 0 --no-cpu > gpurun_out/gx.log 2>gpurun_out/gx.err || { echo "$lib failed"; tail -5 gpurun_out/gx.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/gx.log')); print(sys.argv[1], d['ms_per_step'], d['p50_batch_ms'])" $lib
done
