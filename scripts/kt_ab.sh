# Kernel-trace A/B of library variants (run on the GPU box):
#   bash scripts/kt_ab.sh CONFIG name...   ("base": the product library,
#   others scripts/micro/var/libfdbcs_NAME.so).  Summaries: gpurun_out/ktab/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=$1; shift
O=gpurun_out/ktab
mkdir -p $O
mark=k_live_ingest; [ "$cfg" = 5 ] && mark="k_ingest<"
for v in "$@"; do
  if [ "$v" = base ]; then unset FDBCS_LIB_PATH; else export FDBCS_LIB_PATH=$PWD/scripts/micro/var/libfdbcs_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- \
    python3 -u bench.py --config $cfg --no-cpu --no-shim --lm-batches 0 --stage-batches 0 --latency-batches 0 \
    --steps ${STEPS:-50} --warmup ${WARMUP:-5} > $O/${cfg}_${v}.log 2>&1 || { echo "$v kernel trace failed"; tail -5 $O/${cfg}_${v}.log; exit 1; }
  kt=$(find $O/kt_$v -name "*kernel_trace.csv" | head -1)
  python3 scripts/prof_summary.py "$kt" $(( ${STEPS:-50} - 1 )) "$mark" > $O/${cfg}_${v}.txt 2>&1
  rm -rf $O/kt_$v
  echo "== $v"; head -${TOP:-12} $O/${cfg}_${v}.txt
done
