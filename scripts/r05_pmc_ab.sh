# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and kernel times of
# library variants on the bench workload (run on the GPU box):
#   bash scripts/r05_pmc_ab.sh CONFIG name...
# name "base" = the product library; others = scripts/micro/var/libfdbcs_NAME.so
# (scripts/build_variants.sh).  Summaries: gpurun_out/r05ab/NAME_{pmc,kt}.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=$1; shift
O=gpurun_out/r05ab
mkdir -p $O
common="--config $cfg --no-cpu --no-shim --lm-batches 0 --stage-batches 0 --latency-batches 0"
for v in "$@"; do
  if [ "$v" = base ]; then unset FDBCS_LIB_PATH; else export FDBCS_LIB_PATH=$PWD/scripts/micro/var/libfdbcs_$v.so; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    FDBCS_LIVE=0 timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_$v/p_$ctr -o run -- \
      python3 -u bench.py $common --steps ${STEPS:-50} --warmup 5 > $O/${v}_pmc_$ctr.log 2>&1 || { echo "$v pmc $ctr failed"; tail -5 $O/${v}_pmc_$ctr.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $O/pmc_$v $(( ${STEPS:-50} - 1 )) k_ingest > $O/${v}_pmc.txt 2>&1
  rm -rf $O/pmc_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- \
    python3 -u bench.py $common --steps ${STEPS:-50} --warmup 5 > $O/${v}_kt.log 2>&1 || { echo "$v kernel trace failed"; tail -5 $O/${v}_kt.log; exit 1; }
  kt=$(find $O/kt_$v -name "*kernel_trace.csv" | head -1)
  python3 scripts/prof_summary.py "$kt" ${STEPS:-50} k_live_ingest > $O/${v}_kt.txt 2>&1
  rm -rf $O/kt_$v
  echo "$v ok"; head -8 $O/${v}_pmc.txt
done
