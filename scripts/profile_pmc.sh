# HBM traffic counters of the bench workload, one rocprofv3 --pmc pass per
# counter group (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate
# passes).  Run on the GPU box:
#   OUT=pmc bash scripts/profile_pmc.sh FETCH_SIZE WRITE_SIZE -- [bench args...]
# Summary: python scripts/pmc_summary.py gpurun_out/pmc
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-pmc}
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out/$OUT
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  ctrs=$(echo $grp | tr ',' ' ')
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/$OUT/p$i -o run -- \
    python3 -u bench.py --no-cpu --lm-batches 0 "$@" > gpurun_out/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$OUT/p$i.log; exit 1; }
  echo "pass $i ($ctrs) ok"
done
