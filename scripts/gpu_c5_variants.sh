# Config 5 stage timings for library variants (scripts/micro/var/*.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in scripts/micro/var/*.so; do
  FDBCS_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --config 5 --steps 3 --pcie-batches 0 --no-cpu > gpurun_out/var5.log 2>gpurun_out/var5.err || { echo "$lib failed"; tail -5 gpurun_out/var5.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/var5.log')); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r['stage_us'])" $lib
done
